"""BERTSQuAD (Py/tfpark/text/estimator/bert_squad.py:20-102): sequence output ->
Dense(2) -> (start_logits, end_logits); loss = mean of the start / end position
cross-entropies; predictions are ``{"unique_ids", "start_logits", "end_logits"}``."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.tfpark.text.estimator.bert_base import BERTBaseEstimator, BertConfig


class _SpanHead(nn.Module):
    def __init__(self, hidden):
        super().__init__()
        self.w = nn.Parameter(torch.empty(2, hidden).normal_(0.0, 0.02))
        self.b = nn.Parameter(torch.zeros(2))

    def forward(self, seq, pooled, features):
        logits = ops.linear(seq, self.w, self.b).float()     # [B, L, 2]
        out = {"start_logits": logits[..., 0], "end_logits": logits[..., 1]}
        if "unique_ids" in features:
            out["unique_ids"] = features["unique_ids"]
        return out


class BERTSQuAD(BERTBaseEstimator):
    def __init__(self, bert_config_file, init_checkpoint=None, use_one_hot_embeddings=False, optimizer=None,
                 model_dir=None):
        cfg = bert_config_file if isinstance(bert_config_file, BertConfig) else \
            BertConfig.from_json_file(bert_config_file)
        super().__init__(_SpanHead(cfg.hidden_size), cfg, init_checkpoint, use_one_hot_embeddings, optimizer,
                         model_dir)

    def _loss(self, out, labels):
        s = F.cross_entropy(out["start_logits"], labels["start_positions"].long().reshape(-1))
        e = F.cross_entropy(out["end_logits"], labels["end_positions"].long().reshape(-1))
        return (s + e) / 2.0

    def _predict(self, out, features):
        return {k: v for k, v in out.items()}
