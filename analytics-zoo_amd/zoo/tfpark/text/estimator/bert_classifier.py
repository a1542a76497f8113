"""BERTClassifier (Py/tfpark/text/estimator/bert_classifier.py:20-82): pooled
output -> dropout(0.1 in training) -> Dense(num_classes); softmax cross-entropy;
predictions are class probabilities."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.tfpark.text.estimator.bert_base import BERTBaseEstimator


class _ClassifierHead(nn.Module):
    def __init__(self, hidden, num_classes):
        super().__init__()
        self.w = nn.Parameter(torch.empty(num_classes, hidden).normal_(0.0, 0.02))
        self.b = nn.Parameter(torch.zeros(num_classes))

    def forward(self, seq, pooled, features):
        x = F.dropout(pooled, 0.1, self.training)
        return ops.linear(x, self.w, self.b).float()


class BERTClassifier(BERTBaseEstimator):
    def __init__(self, num_classes, bert_config_file, init_checkpoint=None, use_one_hot_embeddings=False,
                 optimizer=None, model_dir=None):
        from zoo.tfpark.text.estimator.bert_base import BertConfig
        cfg = bert_config_file if isinstance(bert_config_file, BertConfig) else \
            BertConfig.from_json_file(bert_config_file)
        super().__init__(_ClassifierHead(cfg.hidden_size, num_classes), cfg, init_checkpoint,
                         use_one_hot_embeddings, optimizer, model_dir, num_classes=num_classes)

    def _loss(self, logits, labels):
        return F.cross_entropy(logits, labels.long().reshape(-1))

    def _predict(self, logits, features):
        return torch.softmax(logits, -1)

    def evaluate(self, input_fn, eval_methods=("acc",), steps=None):
        res = super().evaluate(input_fn, (), steps)
        if "acc" in eval_methods or "accuracy" in eval_methods:
            res["acc"] = self._accuracy(input_fn, steps)
        return res

    @torch.no_grad()
    def _accuracy(self, input_fn, steps):
        ok = n = 0
        for i, (feats, labs) in enumerate(input_fn("eval")):
            if steps is not None and i >= steps:
                break
            feats, labs = self._to(feats), self._to(labs)
            ok += int((self.model(feats).argmax(-1) == labs.long().reshape(-1)).sum())
            n += labs.numel()
        return ok / max(n, 1)
