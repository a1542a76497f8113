"""Loss functions (Py/pipeline/api/keras/objectives.py, Zs keras/objectives/*.scala,
ZooClassNLLCriterion.scala:28-197, the string map of KerasUtils.toBigDLCriterion).

Every loss is ``loss(y_pred, y_true) -> scalar`` (mean over the batch unless
``size_average=False``). ``SoftmaxCrossEntropy`` takes raw logits and runs on
the fused native softmax + cross-entropy kernel (one read of the logits,
gradient produced in the same pass).
"""
import torch
import torch.nn.functional as F

from zoo import ops

EPS = 1e-7


def _native(y_pred, y_true, kind, size_average=True, beta=1.0, weight=None):
    """The native one-pass loss+gradient kernel (zoo/ops/pointwise.py, HK20) for fp32/bf16 GPU
    predictions whose target has the same shape; None otherwise."""
    if not (torch.is_tensor(y_pred) and y_pred.is_cuda and torch.is_tensor(y_true) and
            y_true.shape == y_pred.shape and y_pred.numel() > 0):
        return None
    from zoo.ops.pointwise import elementwise_loss
    w = weight if weight is not None else (1.0 / y_pred.numel() if size_average else 1.0)
    # fp32 math like the reference definitions (y_pred.float()): the cast is differentiable
    return elementwise_loss(y_pred.float(), y_true.float(), kind, w, beta)


class LossFunction:
    name = "loss"

    def __call__(self, y_pred, y_true):
        return self.forward(y_pred, y_true)

    def forward(self, y_pred, y_true):
        raise NotImplementedError

    # BigDL Criterion-style entry points
    def backward(self, y_pred, y_true):
        y = y_pred.detach().requires_grad_(True)
        self.forward(y, y_true).backward()
        return y.grad


def _match(y_true, y_pred):
    y_true = y_true.to(y_pred.device)
    if y_true.dtype != y_pred.dtype and y_true.is_floating_point():
        y_true = y_true.to(y_pred.dtype)
    if y_true.dim() == y_pred.dim() - 1:
        y_true = y_true.unsqueeze(-1)
    return y_true


class ClassNLLCriterion(LossFunction):
    """Negative log likelihood with ``padding_value`` targets ignored
    (ZooClassNLLCriterion). ``log_prob_as_input=False`` takes probabilities."""

    def __init__(self, weights=None, size_average=True, log_prob_as_input=True, zero_based_label=True,
                 padding_value=-1):
        self.weights, self.size_average = weights, size_average
        self.log_prob_as_input, self.zero_based_label = log_prob_as_input, zero_based_label
        self.padding_value = padding_value

    def forward(self, y_pred, y_true):
        t = y_true.to(y_pred.device).long().reshape(-1)
        if not self.zero_based_label:
            t = t - 1
        ignore = self.padding_value if self.padding_value >= 0 else -100
        if self.padding_value >= 0 and not self.zero_based_label:
            ignore = self.padding_value - 1
        if not self.log_prob_as_input and self.weights is None and y_pred.is_cuda:
            # one native pass: loss + gradient of -log(clamp(p[label])) (zoo.ops.loss.prob_nll)
            return ops.prob_nll(y_pred.reshape(t.shape[0], -1), t, EPS, ignore, self.size_average)
        logp = y_pred.float() if self.log_prob_as_input else torch.log(torch.clamp(y_pred.float(), EPS, 1.0))
        logp = logp.reshape(t.shape[0], -1)
        w = None if self.weights is None else torch.as_tensor(self.weights, dtype=torch.float32, device=logp.device)
        return F.nll_loss(logp, t, weight=w, ignore_index=ignore, reduction="mean" if self.size_average else "sum")


class SparseCategoricalCrossEntropy(ClassNLLCriterion):
    def __init__(self, log_prob_as_input=False, zero_based_label=True, weights=None, size_average=True,
                 padding_value=-1):
        super().__init__(weights, size_average, log_prob_as_input, zero_based_label, padding_value)


class SoftmaxCrossEntropy(LossFunction):
    """Cross-entropy on raw logits with the fused native kernel."""

    def __init__(self, zero_based_label=True, ignore_index=-100):
        self.zero_based_label, self.ignore_index = zero_based_label, ignore_index

    def forward(self, y_pred, y_true):
        t = y_true.to(y_pred.device).long().reshape(-1)
        if not self.zero_based_label:
            t = t - 1
        return ops.softmax_cross_entropy(y_pred.reshape(t.shape[0], -1), t, self.ignore_index)


class CategoricalCrossEntropy(LossFunction):
    """-sum(y_true * log(y_pred)) with probabilities in and one-hot targets."""

    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred)
        p = torch.clamp(y_pred.float(), EPS, 1.0 - EPS)
        return -(y_true.float() * torch.log(p)).sum(-1).mean()


class BinaryCrossEntropy(LossFunction):
    def __init__(self, weights=None, size_average=True):
        self.weights, self.size_average = weights, size_average

    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred).float()
        p = torch.clamp(y_pred.float(), EPS, 1.0 - EPS)
        if self.weights is None:
            r = _native(y_pred, y_true, "bce", self.size_average)
            if r is not None:
                return r
        w = None if self.weights is None else torch.as_tensor(self.weights, dtype=torch.float32, device=p.device)
        return F.binary_cross_entropy(p, y_true, weight=w, reduction="mean" if self.size_average else "sum")


class MeanSquaredError(LossFunction):
    def __init__(self, size_average=True):
        self.size_average = size_average

    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred)
        r = _native(y_pred, y_true, "mse", self.size_average)
        if r is not None:
            return r
        return F.mse_loss(y_pred.float(), y_true.float(), reduction="mean" if self.size_average else "sum")


class MeanAbsoluteError(LossFunction):
    def __init__(self, size_average=True):
        self.size_average = size_average

    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred)
        r = _native(y_pred, y_true, "mae", self.size_average)
        if r is not None:
            return r
        return F.l1_loss(y_pred.float(), y_true.float(), reduction="mean" if self.size_average else "sum")


class MeanAbsolutePercentageError(LossFunction):
    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred).float()
        r = _native(y_pred, y_true, "mape", True)
        if r is not None:
            return r
        diff = (y_true - y_pred.float()).abs() / torch.clamp(y_true.abs(), EPS, float("inf"))
        return 100.0 * diff.mean()


class MeanSquaredLogarithmicError(LossFunction):
    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred).float()
        r = _native(y_pred, y_true, "msle", True)
        if r is not None:
            return r
        a = torch.log(torch.clamp(y_pred.float(), EPS, float("inf")) + 1.0)
        b = torch.log(torch.clamp(y_true, EPS, float("inf")) + 1.0)
        return ((a - b) ** 2).mean()


class Hinge(LossFunction):
    def __init__(self, margin=1.0, size_average=True):
        self.margin, self.size_average = margin, size_average

    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred).float()
        r = _native(y_pred, y_true, "hinge", self.size_average, self.margin)
        if r is not None:
            return r
        l = torch.clamp(self.margin - y_true * y_pred.float(), min=0)
        return l.mean() if self.size_average else l.sum()


class SquaredHinge(Hinge):
    def __init__(self, margin=1.0, size_average=False):
        super().__init__(margin, size_average)

    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred).float()
        r = _native(y_pred, y_true, "squared_hinge", True, self.margin)
        if r is not None:
            return r
        l = torch.clamp(self.margin - y_true * y_pred.float(), min=0) ** 2
        return l.mean()


class KullbackLeiblerDivergence(LossFunction):
    def forward(self, y_pred, y_true):
        rows = y_pred.numel() // max(y_pred.shape[-1], 1) if y_pred.dim() else 1
        r = _native(y_pred, _match(y_true, y_pred).float(), "kld", True, weight=1.0 / max(rows, 1))
        if r is not None:
            return r
        y_true = torch.clamp(_match(y_true, y_pred).float(), EPS, 1.0)
        y_pred = torch.clamp(y_pred.float(), EPS, 1.0)
        return (y_true * torch.log(y_true / y_pred)).sum(-1).mean()


class CosineProximity(LossFunction):
    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred).float()
        a = F.normalize(y_true, dim=-1)
        b = F.normalize(y_pred.float(), dim=-1)
        return -(a * b).sum(-1).mean()


class Poisson(LossFunction):
    def forward(self, y_pred, y_true):
        y_true = _match(y_true, y_pred).float()
        r = _native(y_pred, y_true, "poisson", True)
        if r is not None:
            return r
        p = y_pred.float()
        return (p - y_true * torch.log(p + EPS)).mean()


class RankHinge(LossFunction):
    """Pairwise ranking hinge: consecutive (positive, negative) rows
    (RankHinge.scala: max(neg - pos + margin, 0))."""

    def __init__(self, margin=1.0):
        self.margin = margin

    def forward(self, y_pred, y_true):
        p = y_pred.float().reshape(-1, 2)
        return torch.clamp(p[:, 1] - p[:, 0] + self.margin, min=0).mean()


class MarginRankingLoss(RankHinge):
    pass


class TorchLoss(LossFunction):
    """Wrap any PyTorch loss module/function (TorchCriterion)."""

    def __init__(self, fn):
        self.fn = fn

    def forward(self, y_pred, y_true):
        return self.fn(y_pred, y_true.to(y_pred.device))


_STRINGS = {
    "binary_crossentropy": BinaryCrossEntropy, "categorical_crossentropy": CategoricalCrossEntropy,
    "mse": MeanSquaredError, "mean_squared_error": MeanSquaredError, "mae": MeanAbsoluteError,
    "mean_absolute_error": MeanAbsoluteError, "hinge": Hinge, "mape": MeanAbsolutePercentageError,
    "mean_absolute_percentage_error": MeanAbsolutePercentageError, "msle": MeanSquaredLogarithmicError,
    "mean_squared_logarithmic_error": MeanSquaredLogarithmicError, "squared_hinge": SquaredHinge,
    "sparse_categorical_crossentropy": SparseCategoricalCrossEntropy, "kld": KullbackLeiblerDivergence,
    "kullback_leibler_divergence": KullbackLeiblerDivergence, "cosine_proximity": CosineProximity,
    "poisson": Poisson, "rank_hinge": RankHinge, "softmax_crossentropy": SoftmaxCrossEntropy,
}


def to_criterion(loss):
    if isinstance(loss, LossFunction):
        return loss
    if isinstance(loss, str):
        k = loss.lower()
        if k not in _STRINGS:
            raise ValueError("Unsupported loss: %s" % loss)
        c = _STRINGS[k]()
        c.name = k
        return c
    if hasattr(loss, "graph"):  # autograd CustomLoss
        return TorchLoss(lambda p, t: loss(p, t))
    if callable(loss):
        return TorchLoss(loss)
    raise TypeError("loss must be a LossFunction, string or callable")


# short keras aliases
mse = MSE = MeanSquaredError
mae = MAE = MeanAbsoluteError
