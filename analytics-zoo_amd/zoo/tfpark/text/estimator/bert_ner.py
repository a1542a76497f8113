"""BERTNER (Py/tfpark/text/estimator/bert_ner.py:20-75): final sequence output ->
dropout -> Dense(num_entities); token-level softmax cross-entropy weighted by
``input_mask``; predictions are per-token argmax labels."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.tfpark.text.estimator.bert_base import BERTBaseEstimator, BertConfig


class _TokenHead(nn.Module):
    def __init__(self, hidden, n_out):
        super().__init__()
        self.w = nn.Parameter(torch.empty(n_out, hidden).normal_(0.0, 0.02))
        self.b = nn.Parameter(torch.zeros(n_out))

    def forward(self, seq, pooled, features):
        x = F.dropout(seq, 0.1, self.training)
        mask = features.get("input_mask")
        return {"logits": ops.linear(x, self.w, self.b).float(),
                "mask": torch.ones(seq.shape[:2], device=seq.device) if mask is None else mask.float()}


class BERTNER(BERTBaseEstimator):
    def __init__(self, num_entities, bert_config_file, init_checkpoint=None, use_one_hot_embeddings=False,
                 optimizer=None, model_dir=None):
        cfg = bert_config_file if isinstance(bert_config_file, BertConfig) else \
            BertConfig.from_json_file(bert_config_file)
        super().__init__(_TokenHead(cfg.hidden_size, num_entities), cfg, init_checkpoint, use_one_hot_embeddings,
                         optimizer, model_dir, num_entities=num_entities)

    def _loss(self, out, labels):
        logits, mask = out["logits"], out["mask"].reshape(-1)
        per = F.cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.long().reshape(-1), reduction="none")
        return (per * mask).sum() / (mask.sum() + 1e-12)

    def _predict(self, out, features):
        return out["logits"].argmax(-1)
