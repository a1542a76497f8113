"""GAN training: GanOptimMethod (Zs/tfpark/GanOptimMethod.scala:26-77) and
GANEstimator (Py/tfpark/gan/gan_estimator.py).

Generator and discriminator parameters live in ONE flat buffer, generator
first (``g_param_size`` elements). Step k updates the discriminator slice if
k mod (d_steps + g_steps) < d_steps, else the generator slice — exactly the
reference's schedule — so gradient all-reduce and the fused optimizer
kernels see a single buffer.
"""
import torch


class GanOptimMethod:
    def __init__(self, d_optim, g_optim, d_steps, g_steps, g_param_size):
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        self.d_optim, self.g_optim = to_optim_method(d_optim), to_optim_method(g_optim)
        self.d_steps, self.g_steps, self.g_param_size = int(d_steps), int(g_steps), int(g_param_size)
        self.state = {"epoch": 1, "neval": 1, "evalCounter": 0}

    def in_d_state(self, nevals=None):
        n = self.state["evalCounter"] if nevals is None else nevals
        return n % (self.d_steps + self.g_steps) < self.d_steps

    def step(self, master, grad, bf16=None, gscale=1.0):
        g = self.g_param_size
        if self.in_d_state():
            self.d_optim.step(master[g:], grad[g:], None if bf16 is None else bf16[g:], gscale)
        else:
            self.g_optim.step(master[:g], grad[:g], None if bf16 is None else bf16[:g], gscale)
        self.state["evalCounter"] += 1
        self.state["neval"] += 1

    def current_lr(self):
        return self.d_optim.current_lr()

    def update_epoch(self, epoch):
        self.state["epoch"] = epoch

    def state_dict(self):
        return {"class": "GanOptimMethod", "state": dict(self.state), "d": self.d_optim.state_dict(),
                "g": self.g_optim.state_dict()}

    def load_state_dict(self, d):
        self.state.update(d.get("state", {}))
        self.d_optim.load_state_dict(d["d"])
        self.g_optim.load_state_dict(d["g"])

    def to(self, device):
        self.d_optim.to(device)
        self.g_optim.to(device)
        return self


class GANEstimator:
    """generator_fn / discriminator_fn: nn.Modules. Losses:
    generator_loss_fn(d_fake_logits) and discriminator_loss_fn(d_real_logits, d_fake_logits)."""

    def __init__(self, generator, discriminator, generator_loss_fn, discriminator_loss_fn, generator_optimizer,
                 discriminator_optimizer, generator_steps=1, discriminator_steps=1, noise_dim=None, device=None):
        from zoo.common.nncontext import get_nncontext
        from zoo.parallel.ddp import GradSync
        from zoo.parallel.flat import FlatParams
        self.device = torch.device(device) if device is not None else get_nncontext().device
        self.G, self.D = generator.to(self.device), discriminator.to(self.device)
        self.g_loss_fn, self.d_loss_fn = generator_loss_fn, discriminator_loss_fn
        self.noise_dim = noise_dim
        g_params = [p for p in self.G.parameters() if p.requires_grad]
        d_params = [p for p in self.D.parameters() if p.requires_grad]
        # FlatParams lays parameters out in REVERSE order: pass D first so G lands first
        self.flat = FlatParams(d_params + g_params, device=self.device, bf16_copy=False)
        n_d = len(d_params)
        g_off = [o for p, o in zip(self.flat.params, self.flat.offsets)]
        g_size = self.flat.offsets[len(g_params)] if n_d else self.flat.numel
        assert all(o < g_size for o in g_off[:len(g_params)])
        self.optim = GanOptimMethod(discriminator_optimizer, generator_optimizer, discriminator_steps,
                                    generator_steps, g_size)
        self.sync = GradSync(self.flat, mode="allreduce", overlap=False)
        self.sync.broadcast_parameters(0)

    def _noise(self, n):
        return torch.randn(n, self.noise_dim, device=self.device)

    def train_step(self, real, noise=None):
        real = real.to(self.device)
        noise = self._noise(real.shape[0]) if noise is None else noise.to(self.device)
        self.flat.grad.zero_()
        fake = self.G(noise)
        if self.optim.in_d_state():
            loss = self.d_loss_fn(self.D(real), self.D(fake.detach()))
        else:
            loss = self.g_loss_fn(self.D(fake))
        loss.backward()
        self.sync.step(self.optim)
        return float(loss)

    def train(self, data, steps):
        losses = []
        it = iter(data)
        for _ in range(steps):
            try:
                batch = next(it)
            except StopIteration:
                it = iter(data)
                batch = next(it)
            real = batch[0] if isinstance(batch, (list, tuple)) else batch
            losses.append(self.train_step(real))
        return losses

    @torch.no_grad()
    def generate(self, n):
        return self.G(self._noise(n)).cpu()
