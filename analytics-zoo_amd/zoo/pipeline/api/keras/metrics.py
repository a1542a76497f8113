"""Validation metrics (Py/pipeline/api/keras/metrics.py; Zs keras/metrics
AUC.scala:36-211, Accuracy.scala:36-117, MAE.scala; Ranker NDCG/MAP,
Zs/models/common/Ranker.scala; BigDL Top1Accuracy/Loss/HitRatio [ext]).

Distributed protocol (replaces the Spark reduce of ValidationResults,
Topology.scala:1459-1519): each metric keeps a small vector of float partial
sums per rank (``new_accumulator``/``update``); the engine all-reduces all
metrics' vectors in ONE collective and calls ``result`` on the sums.
"""
import numpy as np
import torch


class ValidationMethod:
    name = "metric"
    n_acc = 2

    def new_accumulator(self):
        return [0.0] * self.n_acc

    def update(self, acc, output, target, criterion=None):
        raise NotImplementedError

    def result(self, acc):
        return acc[0] / max(acc[1], 1e-12)

    # single-process convenience
    def __call__(self, output, target):
        a = self.new_accumulator()
        self.update(a, output, target)
        return self.result(a)


def _labels(target, zero_based=True):
    t = target.reshape(-1).long()
    return t if zero_based else t - 1


class Top1Accuracy(ValidationMethod):
    name = "Top1Accuracy"

    def __init__(self, zero_based_label=True):
        self.zero_based_label = zero_based_label

    def update(self, acc, output, target, criterion=None):
        out = output.float()
        t = _labels(target.to(out.device), self.zero_based_label)
        if out.dim() == 1 or out.shape[-1] == 1:
            pred = (out.reshape(-1) > 0.5).long()
        else:
            pred = out.reshape(t.shape[0], -1).argmax(-1)
        acc[0] += float((pred == t).sum())
        acc[1] += float(t.shape[0])


class Accuracy(Top1Accuracy):
    name = "Accuracy"


class SparseCategoricalAccuracy(Top1Accuracy):
    name = "SparseCategoricalAccuracy"


class CategoricalAccuracy(ValidationMethod):
    name = "CategoricalAccuracy"

    def update(self, acc, output, target, criterion=None):
        pred = output.float().argmax(-1)
        t = target.to(output.device).float().argmax(-1)
        acc[0] += float((pred == t).sum())
        acc[1] += float(t.numel())


class BinaryAccuracy(ValidationMethod):
    name = "BinaryAccuracy"

    def update(self, acc, output, target, criterion=None):
        pred = (output.float().reshape(-1) > 0.5).float()
        t = target.to(output.device).float().reshape(-1)
        acc[0] += float((pred == t).sum())
        acc[1] += float(t.numel())


class Top5Accuracy(ValidationMethod):
    name = "Top5Accuracy"

    def __init__(self, zero_based_label=True):
        self.zero_based_label = zero_based_label

    def update(self, acc, output, target, criterion=None):
        t = _labels(target.to(output.device), self.zero_based_label)
        top = output.float().reshape(t.shape[0], -1).topk(min(5, output.shape[-1]), dim=-1).indices
        acc[0] += float((top == t.unsqueeze(1)).any(1).sum())
        acc[1] += float(t.shape[0])


ZooTop5Accuracy = Top5Accuracy


class MAE(ValidationMethod):
    name = "MAE"

    def update(self, acc, output, target, criterion=None):
        t = target.to(output.device).float().reshape(output.shape)
        acc[0] += float((output.float() - t).abs().sum())
        acc[1] += float(t.numel())


class Loss(ValidationMethod):
    name = "Loss"

    def __init__(self, criterion=None):
        self.criterion = criterion

    def update(self, acc, output, target, criterion=None):
        crit = self.criterion or criterion
        n = output.shape[0]
        acc[0] += float(crit(output, target.to(output.device))) * n
        acc[1] += float(n)


class AUC(ValidationMethod):
    """Area under ROC with ``threshold_num`` fixed thresholds (AUC.scala:128-211)."""

    name = "AUC"

    def __init__(self, threshold_num=200):
        self.T = int(threshold_num)
        self.n_acc = 2 * self.T

    def update(self, acc, output, target, criterion=None):
        p = output.float().reshape(-1)
        if output.dim() > 1 and output.shape[-1] == 2:
            p = output.float()[:, 1]
        t = target.to(output.device).float().reshape(-1)
        if p.is_cuda and self.T > 1:
            # one native histogram pass (HK14): bin i = [i/(T-1), (i+1)/(T-1)); TP/FP at threshold
            # i are the suffix sums from bin i
            from zoo.ops._native import native
            h = native().auc_hist(p.contiguous(), t.contiguous(), self.T, 0.0, self.T / (self.T - 1.0))
            suf = h.flip(1).cumsum(1).flip(1).double().cpu().numpy()
            for i in range(self.T):
                acc[i] += float(suf[0, i])
                acc[self.T + i] += float(suf[1, i])
            return
        th = torch.linspace(0, 1, self.T, device=p.device)
        predpos = p.unsqueeze(0) >= th.unsqueeze(1)        # [T, n]
        pos = (t > 0.5).unsqueeze(0)
        tp = (predpos & pos).sum(1).float().cpu().numpy()
        fp = (predpos & ~pos).sum(1).float().cpu().numpy()
        for i in range(self.T):
            acc[i] += float(tp[i])
            acc[self.T + i] += float(fp[i])

    def result(self, acc):
        tp = np.asarray(acc[: self.T])
        fp = np.asarray(acc[self.T:])
        P, N = tp[0], fp[0]
        if P == 0 or N == 0:
            return 0.0
        tpr = np.concatenate([tp / P, [0.0]])
        fpr = np.concatenate([fp / N, [0.0]])
        return float(np.sum((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2))


class HitRatio(ValidationMethod):
    """HR@k with one positive followed by ``neg_num`` negatives per group."""

    name = "HitRatio"

    def __init__(self, k=10, neg_num=100):
        self.k, self.neg = k, neg_num

    def update(self, acc, output, target, criterion=None):
        s = output.float().reshape(-1, self.neg + 1)
        rank = (s[:, 1:] > s[:, :1]).sum(1)
        acc[0] += float((rank < self.k).sum())
        acc[1] += float(s.shape[0])


class NDCG(ValidationMethod):
    name = "NDCG"

    def __init__(self, k=10, neg_num=100):
        self.k, self.neg = k, neg_num

    def update(self, acc, output, target, criterion=None):
        s = output.float().reshape(-1, self.neg + 1)
        rank = (s[:, 1:] > s[:, :1]).sum(1).float()
        g = torch.where(rank < self.k, 1.0 / torch.log2(rank + 2.0), torch.zeros_like(rank))
        acc[0] += float(g.sum())
        acc[1] += float(s.shape[0])


class MAP(ValidationMethod):
    name = "MAP"

    def __init__(self, k=10, neg_num=100):
        self.k, self.neg = k, neg_num

    def update(self, acc, output, target, criterion=None):
        s = output.float().reshape(-1, self.neg + 1)
        rank = (s[:, 1:] > s[:, :1]).sum(1).float()
        g = torch.where(rank < self.k, 1.0 / (rank + 1.0), torch.zeros_like(rank))
        acc[0] += float(g.sum())
        acc[1] += float(s.shape[0])


class TreeNNAccuracy(Top1Accuracy):
    name = "TreeNNAccuracy"

    def update(self, acc, output, target, criterion=None):
        out = output[:, 0] if output.dim() == 3 else output
        super().update(acc, out, target.reshape(target.shape[0], -1)[:, 0] if target.dim() > 1 else target)


def _acc_for_loss(criterion):
    n = getattr(criterion, "name", "") or type(criterion).__name__.lower()
    if "sparse" in n or "softmax" in n or "classnll" in n:
        return SparseCategoricalAccuracy()
    if n.startswith("categorical"):
        return CategoricalAccuracy()
    if "binary" in n:
        return BinaryAccuracy()
    return Accuracy()


def to_metrics(metrics, criterion=None):
    """Metric strings -> ValidationMethods (KerasUtils.toBigDLMetrics)."""
    if metrics is None:
        return []
    if isinstance(metrics, (ValidationMethod, str)):
        metrics = [metrics]
    out = []
    for m in metrics:
        if isinstance(m, ValidationMethod):
            out.append(m)
            continue
        k = m.lower()
        if k in ("accuracy", "acc"):
            out.append(_acc_for_loss(criterion))
        elif k in ("top5accuracy", "top5acc"):
            out.append(Top5Accuracy())
        elif k == "mae":
            out.append(MAE())
        elif k == "auc":
            out.append(AUC())
        elif k == "loss":
            out.append(Loss(criterion))
        elif k == "treennaccuracy":
            out.append(TreeNNAccuracy())
        else:
            raise ValueError("Unsupported metric: %s" % m)
    return out
