"""TFOptimizer / TFEstimator / ZooOptimizer (Py/tfpark/tf_optimizer.py, estimator.py,
zoo_optimizer.py) on the TrainingEngine."""
import torch

from zoo.common import triggers as T


class ZooOptimizer:
    """Wraps an optimizer spec so gradients are aggregated by the engine (zoo_optimizer.py:20-81)."""

    def __init__(self, optimizer="adam"):
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        self.optim = to_optim_method(optimizer)


class TFOptimizer:
    def __init__(self, model, optim_method=None, dataset=None, clip=None):
        self.model, self.dataset = model, dataset
        if optim_method is not None:
            from zoo.pipeline.api.keras.optimizers import to_optim_method
            model._optim = to_optim_method(optim_method.optim if isinstance(optim_method, ZooOptimizer)
                                           else optim_method)
            model._engine = None

    @classmethod
    def from_keras(cls, keras_model, dataset, optim_method=None, val_split=0.0, **kwargs):
        m = keras_model.model if hasattr(keras_model, "model") and hasattr(keras_model, "fit") and \
            not hasattr(keras_model, "_get_engine") else keras_model
        return cls(m, optim_method, dataset)

    @classmethod
    def from_loss(cls, loss, optim_method=None, dataset=None, clip_norm=None, clip_value=None, **kwargs):
        """Train the variables of a TF graph to minimise an in-graph loss tensor
        (tf_optimizer.py from_loss). ``loss`` is a :class:`TFNet` whose single output is
        the loss and whose inputs are the placeholders the dataset feeds (features and
        labels); its variables must be trainable. The graph runs on the TF-graph executor,
        its gradient comes from autograd through the executed ops, and the update is the
        fused native optimizer over the flat parameter buffer."""
        return _GraphLossOptimizer(loss, optim_method or "adam", dataset, clip_norm, clip_value)

    @classmethod
    def from_train_op(cls, train_op, loss, dataset=None, **kwargs):
        """In-graph training op (tf_optimizer.py from_train_op): ``loss`` is the TFNet of
        the loss; ``train_op`` names the op (usually the NoOp grouping the updates) of an
        optimizer in the same graph. Its Apply* ops give the optimizer and its constant
        hyper-parameters (GradientDescent, Momentum, Adam, Adagrad, RMSProp), which are run
        as the equivalent native optimizer on the same variables."""
        return _GraphLossOptimizer(loss, _optim_from_train_op(loss, train_op), dataset, None, None)

    def set_constant_gradient_clipping(self, min_value, max_value):
        self.model.set_constant_gradient_clipping(min_value, max_value)

    def set_gradient_clipping_by_l2_norm(self, clip_norm):
        self.model.set_gradient_clipping_by_l2_norm(clip_norm)

    def set_train_summary(self, summary):
        self.model._tb = (summary, self.model._tb[1] if self.model._tb else summary)

    def optimize(self, end_trigger=None, checkpoint_trigger=None):
        eng = self.model._get_engine()
        eng.fit(self.dataset.get_training_data(), end_trigger=end_trigger or T.MaxEpoch(1),
                validation=self.dataset.get_validation_data(), val_methods=self.model._metrics or None)
        return self


class TFEstimatorSpec:
    def __init__(self, mode, predictions=None, loss=None):
        self.mode, self.predictions, self.loss = mode, predictions, loss


class TFEstimator:
    """``model_fn(features, labels, mode, params)`` returns a TFEstimatorSpec whose
    ``loss`` is a torch scalar (train/eval) and ``predictions`` a tensor. The
    module(s) it uses are passed as ``modules`` so their parameters are optimized."""

    def __init__(self, model_fn, modules, optimizer="adam", model_dir=None, params=None):
        from zoo.parallel.flat import FlatParams
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        from zoo.common.nncontext import get_nncontext
        self.model_fn, self.params = model_fn, params or {}
        self.modules = torch.nn.ModuleList(modules)
        self.device = get_nncontext().device
        self.modules.to(self.device)
        self.flat = FlatParams(list(self.modules.parameters()), device=self.device,
                               bf16_copy=self.device.type == "cuda")
        self.optim = to_optim_method(optimizer)

    @classmethod
    def from_model_fn(cls, model_fn, modules, optimizer="adam", model_dir=None, params=None):
        return cls(model_fn, modules, optimizer, model_dir, params)

    def train(self, input_fn, steps=None):
        n = 0
        self.modules.train()
        while steps is None or n < steps:
            for x, y in input_fn():
                self.flat.grad.zero_()
                spec = self.model_fn(x.to(self.device), y.to(self.device), "train", self.params)
                spec.loss.backward()
                self.optim.step(self.flat.master, self.flat.grad, self.flat.bf16, 1.0)
                n += 1
                if steps is not None and n >= steps:
                    break
            if steps is None:
                break
        return self

    @torch.no_grad()
    def evaluate(self, input_fn, eval_methods=None):
        self.modules.eval()
        tot, cnt = 0.0, 0
        for x, y in input_fn():
            spec = self.model_fn(x.to(self.device), y.to(self.device), "eval", self.params)
            tot += float(spec.loss) * x.shape[0]
            cnt += x.shape[0]
        return {"loss": tot / max(cnt, 1)}

    @torch.no_grad()
    def predict(self, input_fn):
        self.modules.eval()
        out = []
        for batch in input_fn():
            x = batch[0] if isinstance(batch, (list, tuple)) else batch
            out.append(self.model_fn(x.to(self.device), None, "infer", self.params).predictions.cpu())
        return torch.cat(out).numpy()


def _const_value(net, name):
    from zoo.pipeline.api.net.tf_graph import split_name
    node = net._graph.nodes[split_name(name)[0]]
    while node.op in ("Identity", "ReadVariableOp") and node.inputs:
        node = net._graph.nodes[split_name(node.inputs[0])[0]]
    if node.op != "Const":
        raise ValueError("from_train_op: hyper-parameter %s is not a constant (%s)" % (name, node.op))
    return float(node.attr.get("value").reshape(-1)[0])


def _optim_from_train_op(net, train_op):
    """Walk the train op's inputs (incl. control inputs) to its Apply* / ResourceApply* ops."""
    from zoo.pipeline.api.keras import optimizers as O
    from zoo.pipeline.api.net.tf_graph import split_name
    nodes = net._graph.nodes
    seen, stack, applies = set(), [split_name(train_op.lstrip("^"))[0]], []
    while stack:
        n = stack.pop()
        if n in seen or n not in nodes:
            continue
        seen.add(n)
        node = nodes[n]
        op = node.op.replace("Resource", "")
        if op.startswith("Apply"):
            applies.append((op, node))
            continue
        for i in list(node.inputs) + list(node.controls):
            stack.append(split_name(i.lstrip("^"))[0])
    if not applies:
        raise ValueError("from_train_op: no Apply* update op reachable from %s" % train_op)
    kinds = {op for op, _ in applies}
    if len(kinds) != 1:
        raise NotImplementedError("from_train_op: mixed optimizers %s" % sorted(kinds))
    op, node = applies[0]
    ins = node.inputs
    if op == "ApplyGradientDescent":           # var, alpha, delta
        return O.SGD(learningrate=_const_value(net, ins[1]))
    if op == "ApplyMomentum":                  # var, accum, lr, grad, momentum
        return O.SGD(learningrate=_const_value(net, ins[2]), momentum=_const_value(net, ins[4]),
                     nesterov=bool(node.attr.get("use_nesterov", False)), dampening=0.0)
    if op == "ApplyAdam":                      # var, m, v, beta1_power, beta2_power, lr, beta1, beta2, eps, grad
        return O.Adam(lr=_const_value(net, ins[5]), beta_1=_const_value(net, ins[6]),
                      beta_2=_const_value(net, ins[7]), epsilon=_const_value(net, ins[8]))
    if op == "ApplyAdagrad":                   # var, accum, lr, grad
        return O.Adagrad(learningrate=_const_value(net, ins[2]))
    if op == "ApplyRMSProp":                   # var, ms, mom, lr, rho, momentum, epsilon, grad
        return O.RMSprop(learningrate=_const_value(net, ins[3]), decayrate=_const_value(net, ins[4]),
                         epsilon=_const_value(net, ins[6]))
    raise NotImplementedError("from_train_op: %s" % op)


class _GraphLossOptimizer:
    def __init__(self, net, optim_method, dataset, clip_norm, clip_value):
        from zoo.common.nncontext import get_nncontext
        from zoo.parallel.flat import FlatParams
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        from zoo.tfpark.tfnet import TFNet
        if not isinstance(net, TFNet):
            raise TypeError("from_loss / from_train_op take the loss graph as a TFNet (inputs: the placeholders "
                            "the dataset feeds, output: the loss tensor), got %r" % type(net).__name__)
        self.net, self.dataset = net, dataset
        params = [p for p in net.parameters() if p.requires_grad]
        if not params:
            raise ValueError("the loss graph has no trainable variables (build the TFNet with trainable=True)")
        self.device = get_nncontext().device
        net.to(self.device)
        self.flat = FlatParams(params, device=self.device, bf16_copy=False)
        self.optim = to_optim_method(optim_method.optim if isinstance(optim_method, ZooOptimizer) else optim_method)
        self.clip_norm, self.clip_value = clip_norm, clip_value
        self.losses = []

    def _batches(self):
        ds = self.dataset
        data = ds.get_training_data() if hasattr(ds, "get_training_data") else ds
        for b in data:
            yield [torch.as_tensor(t).to(self.device) for t in (b if isinstance(b, (list, tuple)) else [b])]

    def optimize(self, end_trigger=None, checkpoint_trigger=None):
        epochs = getattr(end_trigger, "max_epoch", None) or getattr(end_trigger, "max", None) or 1
        for _ in range(int(epochs)):
            for batch in self._batches():
                self.flat.grad.zero_()
                loss = self.net(*batch)
                loss = loss.float().mean()
                loss.backward()
                g = self.flat.grad
                if self.clip_value is not None:
                    g.clamp_(-float(self.clip_value), float(self.clip_value))
                if self.clip_norm is not None:
                    n = float(g.norm())
                    if n > self.clip_norm:
                        g.mul_(self.clip_norm / n)
                self.optim.step(self.flat.master, g, None, 1.0)
                self.losses.append(float(loss.detach()))
        return self

