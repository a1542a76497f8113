"""Optimization methods and learning-rate schedules.

API parity with the reference:
  * Zoo ``Adam`` with bias correction + ``PolyEpochDecay``
    (Zs/pipeline/api/keras/optimizers/Adam.scala:38-147, Py/pipeline/api/keras/optimizers.py)
  * ``AdamWeightDecay`` (BERT-style warmup linear/cosine/constant;
    AdamWeightDecay.scala:40-155)
  * BigDL ``SGD`` (momentum, dampening, nesterov, weight decay, lr decay,
    schedules), ``RMSprop``, ``Adagrad``, ``Adadelta``, ``Adamax`` [ext]
  * the Keras string map ``sgd/rmsprop/adamax/adagrad/adadelta/adam``
    (KerasUtils.scala:206-217)

Every method updates a :class:`zoo.parallel.flat.FlatParams` (or a shard of
it) with ONE fused native kernel launch on the GPU — master fp32 weights,
optimizer state and the bf16 compute copy are all written in that pass —
and with the equivalent PyTorch math on the CPU.
"""
import math

import torch

from zoo.ops._native import native


# ----------------------------------------------------------------------------
# learning-rate schedules (BigDL LearningRateSchedule semantics)
# ----------------------------------------------------------------------------
class LearningRateSchedule:
    def rate(self, base_lr, state):
        raise NotImplementedError


class Default(LearningRateSchedule):
    """lr / (1 + neval * learning_rate_decay)"""

    def rate(self, base_lr, state):
        return base_lr / (1.0 + state["neval_prev"] * state.get("lr_decay", 0.0))


class Poly(LearningRateSchedule):
    """lr * (1 - iter/max_iteration) ^ power"""

    def __init__(self, power, max_iteration):
        self.power, self.max_iteration = power, max_iteration

    def rate(self, base_lr, state):
        it = state["neval_prev"]
        if it > self.max_iteration:
            return 0.0
        return base_lr * (1.0 - it / self.max_iteration) ** self.power


class Step(LearningRateSchedule):
    def __init__(self, step_size, gamma):
        self.step_size, self.gamma = step_size, gamma

    def rate(self, base_lr, state):
        return base_lr * self.gamma ** (state["neval_prev"] // self.step_size)


class MultiStep(LearningRateSchedule):
    def __init__(self, step_sizes, gamma):
        self.step_sizes, self.gamma = list(step_sizes), gamma

    def rate(self, base_lr, state):
        k = sum(1 for s in self.step_sizes if state["neval_prev"] >= s)
        return base_lr * self.gamma ** k


class Exponential(LearningRateSchedule):
    def __init__(self, decay_step, decay_rate, stair_case=False):
        self.decay_step, self.decay_rate, self.stair_case = decay_step, decay_rate, stair_case

    def rate(self, base_lr, state):
        p = state["neval_prev"] / self.decay_step
        if self.stair_case:
            p = math.floor(p)
        return base_lr * self.decay_rate ** p


class EpochStep(LearningRateSchedule):
    def __init__(self, step_size, gamma):
        self.step_size, self.gamma = step_size, gamma

    def rate(self, base_lr, state):
        return base_lr * self.gamma ** ((state["epoch"] - 1) // self.step_size)


class EpochDecay(LearningRateSchedule):
    def __init__(self, decay_fn):
        self.decay_fn = decay_fn

    def rate(self, base_lr, state):
        return base_lr * 0.1 ** self.decay_fn(state["epoch"])


class PolyEpochDecay(LearningRateSchedule):
    """init_lr * (1 - epoch/max_epochs) ^ power (Adam.scala:135-147)."""

    def __init__(self, power, max_epochs):
        self.power, self.max_epochs = power, max_epochs

    def rate(self, base_lr, state):
        e = state["epoch"]
        if e >= self.max_epochs:
            return 0.0
        return base_lr * (1.0 - e / self.max_epochs) ** self.power


class Warmup(LearningRateSchedule):
    """lr + delta * iteration (used inside SequentialSchedule)."""

    def __init__(self, delta):
        self.delta = delta

    def rate(self, base_lr, state):
        return base_lr + self.delta * state["neval_prev"]


class EpochDecayWithWarmUp(LearningRateSchedule):
    """BigDL schedule used by the ResNet ImageNet example: linear warmup over
    ``warmup_iteration`` then step decay by epoch through ``decay_type``."""

    def __init__(self, warmup_iteration, warmup_delta, decay_type):
        self.warmup_iteration, self.warmup_delta, self.decay_type = warmup_iteration, warmup_delta, decay_type

    def rate(self, base_lr, state):
        it = state["neval_prev"]
        if it < self.warmup_iteration:
            return base_lr + self.warmup_delta * it
        peak = base_lr + self.warmup_delta * self.warmup_iteration
        return peak * 0.1 ** self.decay_type(state["epoch"])


class SequentialSchedule(LearningRateSchedule):
    def __init__(self, iteration_per_epoch=1):
        self.iteration_per_epoch = iteration_per_epoch
        self.schedules = []

    def add(self, schedule, max_iteration):
        self.schedules.append((schedule, max_iteration))
        return self

    def rate(self, base_lr, state):
        it = state["neval_prev"]
        start = 0
        cur_lr = base_lr
        for sch, n in self.schedules:
            if it < start + n:
                s = dict(state)
                s["neval_prev"] = it - start
                return sch.rate(cur_lr, s)
            s = dict(state)
            s["neval_prev"] = n
            cur_lr = sch.rate(cur_lr, s)
            start += n
        return cur_lr


class Plateau(LearningRateSchedule):
    """Reduce lr when a monitored score stops improving."""

    def __init__(self, monitor="score", factor=0.1, patience=10, mode="min", epsilon=1e-4, cooldown=0,
                 min_lr=0.0):
        self.monitor, self.factor, self.patience, self.mode = monitor, factor, patience, mode
        self.epsilon, self.cooldown, self.min_lr = epsilon, cooldown, min_lr
        self.best = None
        self.wait = 0
        self.cool = 0
        self.scale = 1.0
        self._last_epoch = None

    def rate(self, base_lr, state):
        e = state["epoch"]
        cur = state.get(self.monitor)
        if cur is not None and e != self._last_epoch:
            self._last_epoch = e
            better = self.best is None or (cur < self.best - self.epsilon if self.mode == "min"
                                           else cur > self.best + self.epsilon)
            if better:
                self.best, self.wait = cur, 0
            elif self.cool > 0:
                self.cool -= 1
            else:
                self.wait += 1
                if self.wait >= self.patience:
                    self.scale *= self.factor
                    self.wait, self.cool = 0, self.cooldown
        return max(base_lr * self.scale, self.min_lr)


# ----------------------------------------------------------------------------
# optim methods
# ----------------------------------------------------------------------------
class OptimMethod:
    """Base class. ``state`` mirrors BigDL's OptimMethod Table (epoch, neval, ...)."""

    n_states = 0

    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, weightdecay=0.0, schedule=None):
        self.learning_rate = float(learningrate)
        self.learning_rate_decay = float(learningrate_decay)
        self.weight_decay = float(weightdecay)
        self.schedule = schedule or Default()
        self.state = {"epoch": 1, "neval": 1, "evalCounter": 0, "lr_decay": self.learning_rate_decay}
        self._buffers = None
        self._key = None

    # -- lr ----------------------------------------------------------------
    def current_lr(self):
        s = dict(self.state)
        s["neval_prev"] = self.state["neval"] - 1
        return self.schedule.rate(self.learning_rate, s)

    def get_learningrate(self):
        return self.current_lr()

    # -- state buffers -------------------------------------------------------
    def _ensure_buffers(self, n, device):
        key = (n, str(device))
        if self._key != key:
            self._buffers = [torch.zeros(n, dtype=torch.float32, device=device) for _ in range(self.n_states)]
            self._key = key
        return self._buffers

    # optimizers whose native step clears the gradient after reading it when asked (zero_grad)
    _native_zero_grad = False

    # -- device hyper-parameters (hipGraph-captured updates) --------------------
    # A captured optimizer kernel would replay the learning rate / bias corrections of the
    # capture step. With ``enable_device_hparams`` the native kernels read them from a device
    # [lr, bc1, bc2, first_step] buffer that ``stage_device_hparams`` refreshes (one async
    # host->device copy on the current stream) before each step, captured or eager.
    _dev_hp = None

    def _hparams(self):
        """[lr, bc1, bc2, first_step] of the upcoming step (the kernels' per-step scalars)."""
        return [self.current_lr(), 1.0, 1.0, 0.0]

    def enable_device_hparams(self, device):
        from zoo.ops.devscalar import DeviceStager
        self._hp_stager = DeviceStager(4, torch.float32, device)
        self._dev_hp = self._hp_stager.dev
        self.stage_device_hparams()

    def stage_device_hparams(self):
        if self._dev_hp is not None:
            self._hp_stager.stage(self._hparams())

    def step(self, master, grad, bf16=None, gscale=1.0, zero_grad=False):
        """Update ``master`` (fp32 flat tensor or shard) in place from ``grad``. With
        ``zero_grad`` the native kernels also clear ``grad`` (returns True when they did)."""
        cleared = self.step_range(master, grad, bf16, gscale, 0, master.numel(), zero_grad)
        self.finish_step(bf16 is not None)
        return cleared

    # in-backward updates (zoo.parallel.ddp.GradSync, world 1): the step as a sequence of
    # element ranges issued while the backward still runs, then one counter bump
    def supports_ranges(self):
        """Elementwise native update: any sub-range of the flat buffers can be stepped alone."""
        return bool(self._native_zero_grad) and getattr(self, "parts", None) is None

    def step_range(self, master, grad, bf16, gscale, lo, hi, zero_grad=False):
        """The update of elements [lo, hi) of this step (no counter bump: ``finish_step``)."""
        bufs = self._ensure_buffers(master.numel(), master.device)
        lr = self.current_lr()
        cleared = False
        full = lo == 0 and hi == master.numel()
        m, g = (master, grad) if full else (master[lo:hi], grad[lo:hi])
        b16 = bf16 if (bf16 is None or full) else bf16[lo:hi]
        bs = bufs if full else [t[lo:hi] for t in bufs]
        if master.is_cuda:
            hp = self._dev_hp if (self._dev_hp is not None and self._dev_hp.device == master.device) else None
            if hp is not None:
                native().optim_device_hparams(hp)
            try:
                if zero_grad and self._native_zero_grad:
                    native().optim_zero_grad(True)
                    try:
                        self._step_native(m, g, b16, bs, lr, float(gscale))
                    finally:
                        native().optim_zero_grad(False)
                    cleared = True
                else:
                    self._step_native(m, g, b16, bs, lr, float(gscale))
            finally:
                if hp is not None:
                    native().optim_device_hparams(None)
        else:
            with torch.no_grad():
                self._step_torch(m, g * gscale, bs, lr)
                if b16 is not None:
                    b16.copy_(m)
        return cleared

    def finish_step(self, had_bf16=True):
        if had_bf16:
            from zoo.ops._kern import bump_weights_epoch
            bump_weights_epoch()   # cached dgrad filter flips are stale now
        self.state["neval"] += 1
        self.state["evalCounter"] += 1

    def optimize(self, flat, gscale=1.0):
        self.step(flat.master, flat.grad, flat.bf16, gscale)

    def update_epoch(self, epoch):
        self.state["epoch"] = epoch

    # -- persistence (optimMethod-<name>.<neval> snapshots) --------------------
    def state_dict(self):
        d = {"class": type(self).__name__, "state": dict(self.state), "hyper": self.hyper()}
        if self._buffers is not None:
            d["buffers"] = [b.detach().cpu() for b in self._buffers]
        return d

    def load_state_dict(self, d):
        self.state.update(d.get("state", {}))
        if "buffers" in d and d["buffers"]:
            self._buffers = [b.clone() for b in d["buffers"]]
            self._key = (self._buffers[0].numel(), "cpu")

    def to(self, device):
        if self._buffers is not None:
            self._buffers = [b.to(device) for b in self._buffers]
            self._key = (self._buffers[0].numel(), str(torch.device(device)))
        return self

    def hyper(self):
        return {"learningrate": self.learning_rate, "weightdecay": self.weight_decay}

    def save(self, path, overwrite=True):
        from zoo.utils.checkpoint import save_object
        save_object(self.state_dict(), path, overwrite)

    @classmethod
    def load(cls, path):
        from zoo.utils.checkpoint import load_object
        d = load_object(path)
        klass = globals()[d["class"]]
        m = klass(**d.get("hyper", {}))
        m.load_state_dict(d)
        return m

    def clear_history(self):
        self._buffers = None
        self._key = None


class SGD(OptimMethod):
    """BigDL SGD: x -= lr * (momentum buffer of (g + wd*x)), with dampening / nesterov."""

    _native_zero_grad = True

    n_states = 1

    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, weightdecay=0.0, momentum=0.0, dampening=None,
                 nesterov=False, leaningrate_schedule=None, learningrate_schedule=None, **kw):
        super().__init__(learningrate, learningrate_decay, weightdecay,
                         learningrate_schedule or leaningrate_schedule)
        self.momentum = float(momentum)
        self.dampening = float(momentum if dampening is None and nesterov else (dampening or 0.0))
        if nesterov:
            self.dampening = 0.0
        self.nesterov = bool(nesterov)

    def hyper(self):
        h = super().hyper()
        h.update(momentum=self.momentum, dampening=self.dampening, nesterov=self.nesterov,
                 learningrate_decay=self.learning_rate_decay)
        return h

    def _hparams(self):
        return [self.current_lr(), 1.0, 1.0, 1.0 if self.state["evalCounter"] == 0 else 0.0]

    def _step_native(self, master, grad, bf16, bufs, lr, gscale):
        first = self.state["evalCounter"] == 0
        native().sgd(master, grad, bufs[0] if self.momentum else None, bf16, lr, self.momentum, self.dampening,
                     self.weight_decay, self.nesterov, gscale, first)

    def _step_torch(self, x, g, bufs, lr):
        g = g.clone()
        if self.weight_decay:
            g.add_(x, alpha=self.weight_decay)
        if self.momentum:
            b = bufs[0]
            if self.state["evalCounter"] == 0:
                b.copy_(g)
            else:
                b.mul_(self.momentum).add_(g, alpha=1 - self.dampening)
            g = g.add(b, alpha=self.momentum) if self.nesterov else b
        x.add_(g, alpha=-lr)


class Adam(OptimMethod):
    """Zoo Adam (bias corrected, Adam.scala:59-106)."""

    _native_zero_grad = True

    n_states = 2

    def __init__(self, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-8, decay=0.0, schedule=None,
                 learningrate=None, **kw):
        super().__init__(learningrate if learningrate is not None else lr, decay, 0.0, schedule)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)

    def hyper(self):
        return {"lr": self.learning_rate, "beta_1": self.beta_1, "beta_2": self.beta_2, "epsilon": self.epsilon,
                "decay": self.learning_rate_decay}

    def _bc(self):
        t = self.state["neval"]
        return 1 - self.beta_1 ** t, 1 - self.beta_2 ** t

    def _hparams(self):
        bc1, bc2 = self._bc()
        return [self.current_lr(), bc1, bc2, 0.0]

    def _step_native(self, master, grad, bf16, bufs, lr, gscale):
        bc1, bc2 = self._bc()
        native().adam(master, grad, bufs[0], bufs[1], bf16, lr, self.beta_1, self.beta_2, self.epsilon, 0.0, bc1,
                      bc2, gscale, False)

    def _step_torch(self, x, g, bufs, lr):
        bc1, bc2 = self._bc()
        m, v = bufs
        m.mul_(self.beta_1).add_(g, alpha=1 - self.beta_1)
        v.mul_(self.beta_2).addcmul_(g, g, value=1 - self.beta_2)
        x.addcdiv_(m, v.sqrt().add_(self.epsilon), value=-lr * math.sqrt(bc2) / bc1)


class AdamWeightDecay(OptimMethod):
    """BERT-style Adam with decoupled weight decay and warmup (AdamWeightDecay.scala:75-124)."""

    _native_zero_grad = True

    n_states = 2

    def __init__(self, lr=1e-3, warmup_portion=-1.0, total=-1, schedule="linear", beta1=0.9, beta2=0.999,
                 epsilon=1e-6, weight_decay=0.01, **kw):
        super().__init__(lr, 0.0, weight_decay, None)
        self.warmup_portion, self.total, self.sched = float(warmup_portion), int(total), schedule
        self.beta1, self.beta2, self.epsilon = float(beta1), float(beta2), float(epsilon)

    def hyper(self):
        return {"lr": self.learning_rate, "warmup_portion": self.warmup_portion, "total": self.total,
                "schedule": self.sched, "beta1": self.beta1, "beta2": self.beta2, "epsilon": self.epsilon,
                "weight_decay": self.weight_decay}

    def _warm(self, x):
        w = self.warmup_portion if self.warmup_portion > 0 else 0.002
        if x < w:
            return x / w
        s = self.sched.lower()
        if s == "cosine":
            return 0.5 * (1.0 + math.cos(math.pi * x))
        if s == "constant":
            return 1.0
        if s == "linear":
            return 1.0 - x
        raise ValueError("Only support cosine|constant|linear schedules")

    def current_lr(self):
        if self.total == -1:
            return self.learning_rate
        t = self.state["evalCounter"]
        lr = self.learning_rate * self._warm(t / self.total)
        return lr * self._warm(t / self.total)

    def _step_native(self, master, grad, bf16, bufs, lr, gscale):
        # update = m/(sqrt(v)+eps) + wd*x ; x -= lr*update  (no bias correction)
        native().adam(master, grad, bufs[0], bufs[1], bf16, lr, self.beta1, self.beta2, self.epsilon,
                      self.weight_decay, 1.0, 1.0, gscale, True)

    def _step_torch(self, x, g, bufs, lr):
        m, v = bufs
        m.mul_(self.beta1).add_(g, alpha=1 - self.beta1)
        v.mul_(self.beta2).addcmul_(g, g, value=1 - self.beta2)
        upd = m / (v.sqrt() + self.epsilon)
        if self.weight_decay > 0:
            upd = upd + self.weight_decay * x
        x.add_(upd, alpha=-lr)


class _Adaptive(OptimMethod):
    _native_zero_grad = True
    kind = 0

    def _native_args(self):
        raise NotImplementedError

    def _hparams(self):
        return [self.current_lr(), self._native_args()[3], 1.0, 0.0]

    def _step_native(self, master, grad, bf16, bufs, lr, gscale):
        rho, rho2, eps, bc1 = self._native_args()
        native().adaptive(master, grad, bufs[0], bufs[1] if len(bufs) > 1 else None, bf16, self.kind, lr, rho,
                          rho2, eps, self.weight_decay, bc1, gscale)


class RMSprop(_Adaptive):
    kind, n_states = 0, 1

    def __init__(self, learningrate=1e-2, learningrate_decay=0.0, decayrate=0.99, epsilon=1e-8, weightdecay=0.0,
                 **kw):
        super().__init__(learningrate, learningrate_decay, weightdecay)
        self.decay_rate, self.epsilon = float(decayrate), float(epsilon)

    def hyper(self):
        return {"learningrate": self.learning_rate, "decayrate": self.decay_rate, "epsilon": self.epsilon}

    def _native_args(self):
        return self.decay_rate, 0.0, self.epsilon, 1.0

    def _step_torch(self, x, g, bufs, lr):
        if self.weight_decay:
            g = g + self.weight_decay * x
        a = bufs[0]
        a.mul_(self.decay_rate).addcmul_(g, g, value=1 - self.decay_rate)
        x.addcdiv_(g, a.sqrt().add_(self.epsilon), value=-lr)


class Adagrad(_Adaptive):
    kind, n_states = 1, 1

    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, weightdecay=0.0, epsilon=1e-10, **kw):
        super().__init__(learningrate, learningrate_decay, weightdecay)
        self.epsilon = float(epsilon)

    def _native_args(self):
        return 0.0, 0.0, self.epsilon, 1.0

    def _step_torch(self, x, g, bufs, lr):
        if self.weight_decay:
            g = g + self.weight_decay * x
        bufs[0].addcmul_(g, g)
        x.addcdiv_(g, bufs[0].sqrt().add_(self.epsilon), value=-lr)


class Adadelta(_Adaptive):
    kind, n_states = 2, 2

    def __init__(self, decayrate=0.9, epsilon=1e-10, learningrate=1.0, **kw):
        super().__init__(learningrate, 0.0, 0.0)
        self.decay_rate, self.epsilon = float(decayrate), float(epsilon)

    def hyper(self):
        return {"decayrate": self.decay_rate, "epsilon": self.epsilon, "learningrate": self.learning_rate}

    def _native_args(self):
        return self.decay_rate, 0.0, self.epsilon, 1.0

    def _step_torch(self, x, g, bufs, lr):
        a, d2 = bufs
        a.mul_(self.decay_rate).addcmul_(g, g, value=1 - self.decay_rate)
        d = (d2 + self.epsilon).sqrt() / (a + self.epsilon).sqrt() * g
        d2.mul_(self.decay_rate).addcmul_(d, d, value=1 - self.decay_rate)
        x.add_(d, alpha=-lr)


class Adamax(_Adaptive):
    kind, n_states = 3, 2

    def __init__(self, learningrate=0.002, beta1=0.9, beta2=0.999, epsilon=1e-38, **kw):
        super().__init__(learningrate, 0.0, 0.0)
        self.beta1, self.beta2, self.epsilon = float(beta1), float(beta2), float(epsilon)

    def hyper(self):
        return {"learningrate": self.learning_rate, "beta1": self.beta1, "beta2": self.beta2,
                "epsilon": self.epsilon}

    def _native_args(self):
        return self.beta1, self.beta2, self.epsilon, 1 - self.beta1 ** self.state["neval"]

    def _step_torch(self, x, g, bufs, lr):
        m, u = bufs
        m.mul_(self.beta1).add_(g, alpha=1 - self.beta1)
        torch.maximum(u * self.beta2, g.abs(), out=u)
        bc1 = 1 - self.beta1 ** self.state["neval"]
        x.addcdiv_(m, u + self.epsilon, value=-lr / bc1)


_STRING_MAP = {
    "sgd": lambda: SGD(learningrate=0.01),
    "rmsprop": lambda: RMSprop(learningrate=0.001, decayrate=0.9),
    "adamax": lambda: Adamax(epsilon=1e-8),
    "adagrad": lambda: Adagrad(learningrate=0.01),
    "adadelta": lambda: Adadelta(decayrate=0.95, epsilon=1e-8),
    "adam": lambda: Adam(),
}


def to_optim_method(o):
    """Keras string -> OptimMethod (KerasUtils.toBigDLOptimMethod, KerasUtils.scala:206-217)."""
    if isinstance(o, OptimMethod):
        return o
    if isinstance(o, str):
        k = o.lower()
        if k not in _STRING_MAP:
            raise ValueError("Unsupported optimizer: %s" % o)
        return _STRING_MAP[k]()
    raise TypeError("optimizer must be an OptimMethod or a string, got %r" % (o,))
