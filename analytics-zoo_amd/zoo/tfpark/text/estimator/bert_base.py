"""BERT estimators' shared machinery (Py/tfpark/text/estimator/bert_base.py:21-126).

The reference builds Google's TF BertModel inside a tf.estimator model_fn. Here
the encoder is the framework's BERT layer (fused QKV MFMA GEMM, flash attention
kernel, native LayerNorm) and training runs on the TrainingEngine (flat fp32
master weights, bf16 compute copies, RCCL gradient all-reduce). A Google BERT
checkpoint (``bert_model.ckpt`` tensor bundle) is read with the safe bundle
reader and mapped onto the layer, so ``init_checkpoint`` works as in the
reference.
"""
import json

import numpy as np
import torch
import torch.nn as nn

from zoo.pipeline.api.keras.layers.self_attention import BERT


class BertConfig:
    """google-research/bert ``bert_config.json`` fields."""

    def __init__(self, vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, hidden_act="gelu", hidden_dropout_prob=0.1,
                 attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
                 initializer_range=0.02, **_ignored):
        self.vocab_size, self.hidden_size = int(vocab_size), int(hidden_size)
        self.num_hidden_layers, self.num_attention_heads = int(num_hidden_layers), int(num_attention_heads)
        self.intermediate_size, self.hidden_act = int(intermediate_size), hidden_act
        self.hidden_dropout_prob = float(hidden_dropout_prob)
        self.attention_probs_dropout_prob = float(attention_probs_dropout_prob)
        self.max_position_embeddings, self.type_vocab_size = int(max_position_embeddings), int(type_vocab_size)
        self.initializer_range = float(initializer_range)

    @classmethod
    def from_dict(cls, d):
        return cls(**d)

    @classmethod
    def from_json_file(cls, path):
        with open(path) as f:
            return cls.from_dict(json.load(f))

    def to_dict(self):
        return dict(self.__dict__)


def build_bert(config):
    """BERT layer from a BertConfig (last block + pooled output; LayerNorm eps as Google BERT)."""
    return BERT(vocab=config.vocab_size, hidden_size=config.hidden_size, n_block=config.num_hidden_layers,
                n_head=config.num_attention_heads, max_position_len=config.max_position_embeddings,
                intermediate_size=config.intermediate_size, hidden_drop=config.hidden_dropout_prob,
                attn_drop=config.attention_probs_dropout_prob, initializer_range=config.initializer_range,
                output_all_block=False, type_vocab_size=config.type_vocab_size, layer_norm_eps=1e-12)


def load_bert_checkpoint(bert, ckpt_prefix, scope="bert"):
    """Copy a Google BERT TF checkpoint (``<prefix>.index`` + data shards) into a
    BERT layer. TF dense kernels are [in, out]; the layer stores [out, in] and
    keeps Q/K/V fused as one [3H, H] projection. Returns the loaded variable names."""
    from zoo.pipeline.api.net.tf_graph import read_tensor_bundle
    v = read_tensor_bundle(ckpt_prefix)
    used = []

    def get(name):
        key = "%s/%s" % (scope, name)
        if key not in v:
            raise KeyError("checkpoint has no variable %s" % key)
        used.append(key)
        return torch.from_numpy(np.asarray(v[key], dtype=np.float32))

    def put(param, value):
        with torch.no_grad():
            param.copy_(value.reshape(param.shape).to(param.dtype))

    put(bert.word, get("embeddings/word_embeddings"))
    put(bert.token_type, get("embeddings/token_type_embeddings"))
    pos = get("embeddings/position_embeddings")
    with torch.no_grad():
        bert.position[:pos.shape[0]].copy_(pos[:bert.position.shape[0]])
    put(bert.emb_ln_g, get("embeddings/LayerNorm/gamma"))
    put(bert.emb_ln_b, get("embeddings/LayerNorm/beta"))
    for i, blk in enumerate(bert.blocks):
        p = "encoder/layer_%d/" % i
        q, k, vv = (get(p + "attention/self/%s/kernel" % n) for n in ("query", "key", "value"))
        put(blk.qkv_w, torch.cat([q.t(), k.t(), vv.t()], 0))
        put(blk.qkv_b, torch.cat([get(p + "attention/self/%s/bias" % n) for n in ("query", "key", "value")]))
        put(blk.proj_w, get(p + "attention/output/dense/kernel").t())
        put(blk.proj_b, get(p + "attention/output/dense/bias"))
        put(blk.ln1_g, get(p + "attention/output/LayerNorm/gamma"))
        put(blk.ln1_b, get(p + "attention/output/LayerNorm/beta"))
        put(blk.fc1_w, get(p + "intermediate/dense/kernel").t())
        put(blk.fc1_b, get(p + "intermediate/dense/bias"))
        put(blk.fc2_w, get(p + "output/dense/kernel").t())
        put(blk.fc2_b, get(p + "output/dense/bias"))
        put(blk.ln2_g, get(p + "output/LayerNorm/gamma"))
        put(blk.ln2_b, get(p + "output/LayerNorm/beta"))
    if "%s/pooler/dense/kernel" % scope in v:
        put(bert.pool_w, get("pooler/dense/kernel").t())
        put(bert.pool_b, get("pooler/dense/bias"))
    return used


class BertEncoder(nn.Module):
    """features dict -> (sequence_output [B, L, H], pooled_output [B, H])."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.bert = build_bert(config)

    def forward(self, features):
        ids = features["input_ids"].long()
        B, L = ids.shape
        tt = features.get("token_type_ids")
        tt = torch.zeros_like(ids) if tt is None else tt.long()
        pos = torch.arange(L, device=ids.device).unsqueeze(0).expand(B, L)
        mask = features.get("input_mask")
        xs = [ids, tt, pos] + ([mask.float()] if mask is not None else [])
        seq, pooled = self.bert.call(xs)
        return seq, pooled


def _as_tensor(v):
    return v if torch.is_tensor(v) else torch.as_tensor(np.asarray(v))


def _collate(items):
    if isinstance(items[0], dict):
        return {k: _collate([it[k] for it in items]) for k in items[0]}
    return torch.stack([_as_tensor(it) for it in items])


def bert_input_fn(data, max_seq_length, batch_size, features=("input_ids", "input_mask", "token_type_ids"),
                  extra_features=None, labels=None, label_size=None, shuffle=True):
    """input_fn(mode) over ``data``: a list (or anything with ``collect()``, e.g. an
    XShards / RDD-like) whose elements are ``(features_dict, label)`` for
    train/eval (label: int, int array, or dict of those) or ``features_dict``
    for prediction. Each feature has length ``max_seq_length``."""
    rows = data.collect() if hasattr(data, "collect") else list(data)
    names = list(features) + list((extra_features or {}).keys())

    def input_fn(mode):
        train = mode == "train"
        order = np.random.permutation(len(rows)) if (train and shuffle) else np.arange(len(rows))
        for s in range(0, len(rows), batch_size):
            chunk = [rows[i] for i in order[s:s + batch_size]]
            if train and len(chunk) < batch_size and s > 0:
                break
            if isinstance(chunk[0], tuple):
                feats = _collate([{k: c[0][k] for k in names if k in c[0]} for c in chunk])
                labs = _collate([c[1] for c in chunk])
                for k in ("input_ids", "input_mask", "token_type_ids"):
                    if k in feats:
                        assert feats[k].shape[1] == max_seq_length, "%s must have length %d" % (k, max_seq_length)
                yield feats, labs
            else:
                yield _collate([{k: c[k] for k in names if k in c} for c in chunk]), None
    return input_fn


class BERTBaseEstimator:
    """Base of the BERT estimators: a ``BertEncoder`` + a task head module; the
    subclass supplies ``_loss(outputs, labels)`` and ``_predict(outputs, features)``; the head
    is called as ``head(sequence_output, pooled_output, features)``."""

    def __init__(self, head, bert_config_file, init_checkpoint=None, use_one_hot_embeddings=False,
                 optimizer=None, model_dir=None, **params):
        from zoo.common.nncontext import get_nncontext
        self.config = bert_config_file if isinstance(bert_config_file, BertConfig) else \
            BertConfig.from_json_file(bert_config_file)
        self.params = dict(params, bert_config_file=bert_config_file, init_checkpoint=init_checkpoint,
                           use_one_hot_embeddings=use_one_hot_embeddings)
        self.encoder = BertEncoder(self.config)
        if init_checkpoint:
            load_bert_checkpoint(self.encoder.bert, init_checkpoint)
        self.head = head
        self.model = _TaskModel(self.encoder, head)
        self.model_dir = model_dir
        self.optimizer = optimizer or "adam"
        self.device = get_nncontext().device
        self._engine = None

    def _get_engine(self):
        if self._engine is None:
            from zoo.pipeline.api.keras.optimizers import to_optim_method
            from zoo.pipeline.engine import TrainingEngine
            self._engine = TrainingEngine(self.model, lambda out, lab: self._loss(out, lab),
                                          to_optim_method(self.optimizer), device=self.device)
            if self.model_dir:
                from zoo.common.triggers import SeveralIteration
                self._engine.set_checkpoint(self.model_dir, SeveralIteration(1000))
        return self._engine

    def _to(self, x):
        from zoo.pipeline.engine import _move
        return _move(x, self.device)

    def train(self, input_fn, steps=None):
        eng = self._get_engine()
        n = 0
        while steps is None or n < steps:
            for feats, labs in input_fn("train"):
                feats, labs = self._to(feats), self._to(labs)
                eng.train_step(feats, labs)
                n += 1
                if steps is not None and n >= steps:
                    break
            if steps is None:
                break
        return self

    @torch.no_grad()
    def evaluate(self, input_fn, eval_methods=("acc",), steps=None):
        self.model.to(self.device).eval()
        tot, cnt, correct = 0.0, 0, 0
        for i, (feats, labs) in enumerate(input_fn("eval")):
            if steps is not None and i >= steps:
                break
            feats, labs = self._to(feats), self._to(labs)
            out = self.model(feats)
            bs = feats["input_ids"].shape[0]
            tot += float(self._loss(out, labs)) * bs
            pred = self._predict(out, feats)
            if torch.is_tensor(labs) and torch.is_tensor(pred) and pred.shape == labs.shape:
                correct += int((pred == labs).sum())
            cnt += bs
        res = {"loss": tot / max(cnt, 1)}
        if "acc" in eval_methods or "accuracy" in eval_methods:
            res["acc"] = correct / max(cnt, 1)
        return res

    @torch.no_grad()
    def predict(self, input_fn):
        self.model.to(self.device).eval()
        outs = []
        for feats, _ in input_fn("infer"):
            feats = self._to(feats)
            p = self._predict(self.model(feats), feats)
            outs.append({k: v.cpu() for k, v in p.items()} if isinstance(p, dict) else p.cpu())
        if isinstance(outs[0], dict):
            return {k: torch.cat([o[k] for o in outs]).numpy() for k in outs[0]}
        return torch.cat(outs).numpy()

    def save(self, path):
        from zoo.utils.checkpoint import save_object
        save_object({k: v.detach().cpu() for k, v in self.model.state_dict().items()}, path, True)

    def load(self, path):
        from zoo.utils.checkpoint import load_object
        self.model.load_state_dict(load_object(path))
        if self._engine is not None:
            self._engine.flat.refresh_bf16()
        return self


class _TaskModel(nn.Module):
    def __init__(self, encoder, head):
        super().__init__()
        self.encoder, self.head = encoder, head

    def forward(self, features):
        seq, pooled = self.encoder(features)
        return self.head(seq, pooled, features)

