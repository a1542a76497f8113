"""Estimator / LocalEstimator / Predictor — the user-facing train/evaluate/
predict front ends over the TrainingEngine.

Reference parity:
  * ``Estimator``      — Zs/pipeline/estimator/Estimator.scala:65-183 (train 118-161,
    evaluate 163-176, clipping 137-150); Python Py/pipeline/estimator/estimator.py:21-150
  * ``LocalEstimator`` — Zs/pipeline/estimator/LocalEstimator.scala:37-300: the batch is
    split into ``thread_num`` slices whose per-slice losses are averaged and whose
    gradients are summed then divided by the slice count (optimize 164-216). On one
    MI355X the slices run back to back on the device and accumulate into the flat
    fp32 gradient buffer (no replica copies: the replicas of the reference only
    existed to give each CPU core its own activations).
  * ``Predictor``      — Zs/pipeline/api/Predictor.scala:37-461: batched distributed
    inference; each rank predicts its shard of the data (the analogue of the
    reference's mapPartitions over a broadcast model) and results can be
    gathered to every rank.
  * per-submodule optimizers (Topology.scala:1131-1152):
    ``optim_methods`` may be a dict {submodule name: OptimMethod}; each method
    owns the contiguous range of the flat parameter buffer holding that
    submodule's parameters (see :class:`MultiOptimMethod`).
"""
import logging
import os

import numpy as np
import torch

from zoo.common import triggers as T

log = logging.getLogger("zoo.estimator")


class MultiOptimMethod:
    """Several OptimMethods over disjoint ranges of one flat parameter buffer."""

    def __init__(self, parts):
        self.parts = parts          # [(name, optim, lo, hi)] with flat-buffer offsets
        self.state = {"epoch": 1, "neval": 1}

    def step(self, master, grad, bf16=None, gscale=1.0, base=0):
        n = master.numel()
        for _, o, lo, hi in self.parts:
            a, b = max(lo - base, 0), min(hi - base, n)
            if a < b:
                o.step(master[a:b], grad[a:b], None if bf16 is None else bf16[a:b], gscale)
        self.state["neval"] += 1

    def step_ranges(self, ranges, master, grad, bf16=None, gscale=1.0):
        """ZeRO-1 shard update: ``ranges`` = [((lo, hi) in shard coordinates or None, optim)]."""
        for r, o in ranges:
            if r is None:
                continue
            a, b = r
            o.step(master[a:b], grad[a:b], None if bf16 is None else bf16[a:b], gscale)
        self.state["neval"] += 1

    def current_lr(self):
        return self.parts[0][1].current_lr() if self.parts else 0.0

    def update_epoch(self, epoch):
        self.state["epoch"] = epoch
        for _, o, _, _ in self.parts:
            o.update_epoch(epoch)

    def state_dict(self):
        return {"class": "MultiOptimMethod", "state": dict(self.state),
                "parts": {name: o.state_dict() for name, o, _, _ in self.parts}}

    def load_state_dict(self, d):
        self.state.update(d.get("state", {}))
        for name, o, _, _ in self.parts:
            if name in d.get("parts", {}):
                o.load_state_dict(d["parts"][name])

    def to(self, device):
        for _, o, _, _ in self.parts:
            o.to(device)
        return self


def _resolve_optim(model, optim_methods, flat):
    from zoo.pipeline.api.keras.optimizers import SGD, to_optim_method
    if optim_methods is None:
        return SGD()
    if not isinstance(optim_methods, dict):
        return to_optim_method(optim_methods)
    mods = dict(model.named_modules())
    index = {id(p): i for i, p in enumerate(flat.params)}
    parts = []
    for name, om in optim_methods.items():
        sub = mods.get(name)
        if sub is None:
            sub = next((m for m in model.modules() if getattr(m, "name", None) == name), None)
        if sub is None:
            raise ValueError("no submodule named %r for the optim method" % name)
        idx = sorted(index[id(p)] for p in sub.parameters() if id(p) in index)
        if not idx:
            continue
        if idx != list(range(idx[0], idx[-1] + 1)):
            raise ValueError("parameters of %r are not contiguous in the flat buffer" % name)
        lo = flat.offsets[idx[0]]
        last = idx[-1]
        hi = flat.offsets[last + 1] if last + 1 < len(flat.offsets) else flat.numel
        parts.append((name, to_optim_method(om), lo, hi))
    covered = sum(hi - lo for _, _, lo, hi in parts)
    total = flat.offsets[-1] + flat.params[-1].numel() if flat.params else 0
    if covered < total:
        log.warning("optim_methods cover %d of %d flat parameters; the rest stay frozen", covered, total)
    return MultiOptimMethod(parts)


def _as_featureset(data, batch_size, shuffle):
    from zoo.feature.common import FeatureSet
    if isinstance(data, FeatureSet):
        return data
    if hasattr(data, "to_featureset"):
        return data.to_featureset(batch_size)
    if isinstance(data, (list, tuple)) and len(data) == 2:
        return FeatureSet.from_ndarrays(data[0], data[1], batch_size, shuffle=shuffle)
    if isinstance(data, torch.utils.data.DataLoader):
        return FeatureSet.from_dataloader(data)
    return data


class Estimator:
    """Distributed train / evaluate over FeatureSets (one process per GPU)."""

    def __init__(self, model, optim_methods=None, model_dir=None):
        from zoo.pipeline.engine import TrainingEngine
        self.model = model
        self.model_dir = model_dir
        self._optim_spec = optim_methods
        self._clip = None
        self._engine = None
        self._engine_cls = TrainingEngine

    # -- clipping (Estimator.scala:137-150) ----------------------------------
    def clear_gradient_clipping(self):
        self._clip = None
        if self._engine is not None:
            self._engine.clip = None

    def set_constant_gradient_clipping(self, min, max):  # noqa: A002 - reference names
        from zoo.parallel.ddp import constant_clip
        self._clip = constant_clip(float(min), float(max))
        if self._engine is not None:
            self._engine.clip = self._clip

    def set_l2_norm_gradient_clipping(self, clip_norm):
        from zoo.parallel.ddp import global_norm_clip
        self._clip = global_norm_clip(float(clip_norm))
        if self._engine is not None:
            self._engine.clip = self._clip

    # -- engine ------------------------------------------------------------------
    def _get_engine(self, criterion):
        from zoo.pipeline.api.keras.objectives import to_criterion
        crit = to_criterion(criterion) if criterion is not None else None
        if self._engine is None:
            from zoo.pipeline.api.keras.optimizers import SGD
            eng = self._engine_cls(self.model, crit, SGD(), clip=self._clip)
            eng.optim = _resolve_optim(self.model, self._optim_spec, eng.flat)
            self._engine = eng
        elif crit is not None:
            self._engine.criterion = crit
        return self._engine

    @property
    def engine(self):
        return self._engine

    def train(self, train_set, criterion, end_trigger=None, checkpoint_trigger=None, validation_set=None,
              validation_method=None, batch_size=32):
        """Estimator.scala:118-161: train until ``end_trigger``; at every
        ``checkpoint_trigger`` save to ``model_dir`` and validate."""
        from zoo.pipeline.api.keras.metrics import to_metrics
        eng = self._get_engine(criterion)
        if self.model_dir is not None:
            eng.set_checkpoint(self.model_dir, checkpoint_trigger or T.EveryEpoch(), overwrite=False)
        data = _as_featureset(train_set, batch_size, True)
        val = _as_featureset(validation_set, batch_size, False) if validation_set is not None else None
        methods = to_metrics(validation_method, eng.criterion) if validation_method is not None else None
        eng.fit(data, end_trigger=end_trigger or T.MaxEpoch(1), validation=val, val_methods=methods,
                val_trigger=checkpoint_trigger)
        return self

    def train_minibatch(self, train_set, criterion, end_trigger=None, checkpoint_trigger=None,
                        validation_set=None, validation_method=None):
        return self.train(train_set, criterion, end_trigger, checkpoint_trigger, validation_set, validation_method)

    def train_imagefeature(self, train_set, criterion, end_trigger=None, checkpoint_trigger=None,
                           validation_set=None, validation_method=None, batch_size=32):
        return self.train(train_set, criterion, end_trigger, checkpoint_trigger, validation_set, validation_method,
                          batch_size)

    def evaluate(self, validation_set, validation_method, batch_size=32):
        """Estimator.scala:163-176; returns {method name: value}."""
        from zoo.pipeline.api.keras.metrics import to_metrics
        eng = self._get_engine(None)
        methods = to_metrics(validation_method, eng.criterion)
        res = eng.evaluate(_as_featureset(validation_set, batch_size, False), methods)
        return dict(res)

    def evaluate_imagefeature(self, validation_set, validation_method, batch_size=32):
        return self.evaluate(validation_set, validation_method, batch_size)

    def evaluate_minibatch(self, validation_set, validation_method):
        return self.evaluate(validation_set, validation_method)


class LocalEstimator:
    """Single-device estimator with the reference's thread-slice semantics."""

    def __init__(self, model, criterion, optim_method, validations=None, thread_num=1, device=None):
        from zoo.common.nncontext import get_nncontext
        from zoo.parallel.flat import FlatParams
        from zoo.pipeline.api.keras.metrics import to_metrics
        from zoo.pipeline.api.keras.objectives import to_criterion
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        if thread_num < 1:
            raise ValueError("the number of threads should >= 1")
        self.device = torch.device(device) if device is not None else get_nncontext().device
        self.model = model.to(self.device)
        self.criterion = to_criterion(criterion)
        self.optim = to_optim_method(optim_method)
        self.validations = to_metrics(validations, self.criterion) if validations else []
        self.thread_num = int(thread_num)
        self.flat = FlatParams(list(self.model.parameters()), device=self.device,
                               bf16_copy=self.device.type == "cuda")

    def _slices(self, n):
        stack, extra = divmod(n, self.thread_num)
        par = extra if stack == 0 else self.thread_num
        out, off = [], 0
        for b in range(par):
            ln = stack + (1 if b < extra else 0)
            out.append((off, ln))
            off += ln
        return out

    @staticmethod
    def _take(x, a, n):
        if isinstance(x, (list, tuple)):
            return [t[a:a + n] for t in x]
        return x[a:a + n]

    def optimize(self, x, y):
        """One iteration (LocalEstimator.scala:164-216); returns the mean slice loss."""
        from zoo.ops import workspace
        x = x.to(self.device) if torch.is_tensor(x) else [t.to(self.device) for t in x]
        y = y.to(self.device)
        n = (x[0] if isinstance(x, (list, tuple)) else x).shape[0]
        sl = self._slices(n)
        self.model.train()
        self.flat.grad.zero_()
        total = 0.0
        workspace.begin_step(self.device)
        try:
            for a, ln in sl:
                xi = self._take(x, a, ln)
                out = self.model(xi) if not isinstance(xi, list) else self.model(xi)
                loss = self.criterion(out, y[a:a + ln])
                (loss / len(sl)).backward()
                total = total + loss.detach()
        finally:
            workspace.end_step()
        self.optim.step(self.flat.master, self.flat.grad, self.flat.bf16, 1.0)
        return float(total) / len(sl)

    def fit(self, train_batches, epochs=1, test_batches=None):
        """LocalEstimator.scala:137-162: ``train_batches`` is a sequence of (x, y) minibatches."""
        losses = []
        for ep in range(epochs):
            for x, y in train_batches:
                losses.append(self.optimize(torch.as_tensor(x) if isinstance(x, np.ndarray) else x,
                                            torch.as_tensor(y) if isinstance(y, np.ndarray) else y))
            self.optim.update_epoch(ep + 2)
            if test_batches is not None and self.validations:
                log.info("epoch %d validation %s", ep + 1, self.validate(test_batches))
        return losses

    @torch.no_grad()
    def validate(self, batches):
        accs = [m.new_accumulator() for m in self.validations]
        self.model.eval()
        for x, y in batches:
            x = torch.as_tensor(x).to(self.device) if not isinstance(x, list) else [torch.as_tensor(t).to(
                self.device) for t in x]
            y = torch.as_tensor(y).to(self.device)
            out = self.model(x)
            for m, a in zip(self.validations, accs):
                m.update(a, out, y, self.criterion)
        self.model.train()
        return [(m.name, m.result(a)) for m, a in zip(self.validations, accs)]


class Predictor:
    """Batched (optionally distributed) inference over a model."""

    def __init__(self, model, batch_per_thread=32, device=None):
        from zoo.common.nncontext import get_nncontext
        ctx = get_nncontext()
        self.ctx = ctx
        self.device = torch.device(device) if device is not None else ctx.device
        self.model = model.to(self.device)
        self.batch = int(batch_per_thread)

    @torch.no_grad()
    def _run(self, x):
        was = self.model.training
        self.model.eval()
        xs = x if isinstance(x, (list, tuple)) else [x]
        xs = [torch.as_tensor(t) for t in xs]
        n = xs[0].shape[0]
        outs = []
        for s in range(0, n, self.batch):
            chunk = [t[s:s + self.batch].to(self.device, non_blocking=True) for t in xs]
            o = self.model(chunk[0] if len(chunk) == 1 else chunk)
            outs.append(o.float().cpu() if torch.is_tensor(o) else [t.float().cpu() for t in o])
        self.model.train(was)
        if not outs:
            return torch.zeros(0)
        if torch.is_tensor(outs[0]):
            return torch.cat(outs)
        return [torch.cat([o[i] for o in outs]) for i in range(len(outs[0]))]

    def predict(self, x, distributed=False):
        """``distributed``: every rank predicts rows rank::world of ``x`` and the
        results are all-gathered back into the original order."""
        world, rank = self.ctx.world_size, self.ctx.rank
        if not distributed or world == 1:
            return self._run(x).numpy()
        xs = x if isinstance(x, (list, tuple)) else [x]
        xs = [torch.as_tensor(t) for t in xs]
        n = xs[0].shape[0]
        mine = [t[rank::world] for t in xs]
        out = self._run(mine[0] if len(mine) == 1 else mine)
        import torch.distributed as dist
        per = (n + world - 1) // world
        pad = torch.zeros((per,) + tuple(out.shape[1:]), dtype=out.dtype)
        pad[: out.shape[0]] = out
        dev_pad = pad.to(self.device)
        parts = [torch.empty_like(dev_pad) for _ in range(world)]
        dist.all_gather(parts, dev_pad)
        full = torch.empty((n,) + tuple(out.shape[1:]), dtype=out.dtype)
        for r in range(world):
            cnt = len(range(r, n, world))
            full[r::world] = parts[r][:cnt].cpu()
        return full.numpy()

    def predict_classes(self, x, zero_based_label=True, distributed=False):
        c = np.argmax(self.predict(x, distributed), axis=-1)
        return c if zero_based_label else c + 1


def save_estimator_model(est, path):
    from zoo.utils.checkpoint import save_object
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    save_object({k: v.detach().cpu() for k, v in est.model.state_dict().items()}, path, True)
