"""BERT-base-width numerics on the GPU: the native bf16 BERT (768 wide, 12 heads, 3072 FFN,
sequence 128) with every round-3/4 fusion on -- the LayerNorm residual-gradient add, the GELU
backward in the next linear's dgrad epilogue, the workspace-arena bias-gradient sums, the flash
attention with the additive key mask -- against a plain PyTorch fp32 transcription of the same
network from the same weights:

  * per-parameter-group gradient cosine >= 0.99 after one forward/backward
    (Zs/pipeline/api/keras/layers/BERT.scala:66-402, TransformerLayer.scala:120-181);
  * a 30-step training loss trajectory (SGD + momentum through TrainingEngine, fp32 master
    weights) within 0.02 of the fp32 model trained with torch.optim.SGD.
Dropout is 0 so the two runs see the same function.
"""
import copy
import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

H, NH, INTER, L, B, NBLK, VOCAB = 768, 12, 3072, 128, 8, 12, 2000


class _Cls(nn.Module):
    def __init__(self, bert):
        super().__init__()
        self.bert = bert
        self.fc = nn.Linear(H, 4)

    def forward(self, xs):
        return self.fc(self.bert(xs)[1].float())


def _ref_forward(m, xs):
    """fp32 transcription of zoo BERT + classifier, reading m's (fp32) parameters."""
    bt = m.bert
    tok, typ, pos, am = xs[0].long(), xs[1].long(), xs[2].long(), xs[3]
    eps = bt.layer_norm_eps
    x = F.layer_norm(bt.word[tok] + bt.token_type[typ] + bt.position[pos], (H,), bt.emb_ln_g, bt.emb_ln_b, eps)
    mask = ((1.0 - am.float()) * -10000.0)[:, None, None, :]
    hd = H // NH
    for blk in bt.blocks:
        qkv = (x @ blk.qkv_w.t() + blk.qkv_b).reshape(B, L, 3, NH, hd).permute(2, 0, 3, 1, 4)
        s = qkv[0] @ qkv[1].transpose(-1, -2) / math.sqrt(hd) + mask
        a = (torch.softmax(s, -1) @ qkv[2]).transpose(1, 2).reshape(B, L, H)
        n = F.layer_norm(a @ blk.proj_w.t() + blk.proj_b + x, (H,), blk.ln1_g, blk.ln1_b, eps)
        f = F.gelu(n @ blk.fc1_w.t() + blk.fc1_b) @ blk.fc2_w.t() + blk.fc2_b
        x = F.layer_norm(f + n, (H,), blk.ln2_g, blk.ln2_b, eps)
    pooled = torch.tanh(x[:, 0] @ bt.pool_w.t() + bt.pool_b)
    return m.fc(pooled)


def _setup(gpu, seed=0):
    from zoo.pipeline.api.keras.layers import BERT
    torch.manual_seed(seed)
    bert = BERT(vocab=VOCAB, hidden_size=H, n_block=NBLK, n_head=NH, max_position_len=512, intermediate_size=INTER,
                hidden_drop=0.0, attn_drop=0.0, output_all_block=False)
    m = _Cls(bert)
    g = torch.Generator(device=gpu)
    g.manual_seed(1)
    am = torch.ones(B, L, device=gpu)
    am[:, 100:] = 0.0          # padded tail on every sequence: the key mask is live
    xs = [torch.randint(0, VOCAB, (B, L), device=gpu, generator=g), torch.randint(0, 2, (B, L), device=gpu, generator=g),
          torch.arange(L, device=gpu).repeat(B, 1), am]
    y = torch.randint(0, 4, (B,), device=gpu, generator=g)
    return m, xs, y


def _cos(a, b):
    return F.cosine_similarity(a.double().flatten(), b.double().flatten(), dim=0).item()


def test_bert_base_width_gradients_match_fp32(gpu):
    from zoo.ops import softmax_cross_entropy
    m, xs, y = _setup(gpu)
    nat = copy.deepcopy(m).to(gpu).train()
    ref = copy.deepcopy(m).to(gpu).train()
    ln = softmax_cross_entropy(nat(xs), y)
    ln.backward()
    lr = F.cross_entropy(_ref_forward(ref, xs), y)
    lr.backward()
    assert abs(ln.float().item() - lr.item()) < 0.02, (ln.item(), lr.item())
    rg = dict(ref.named_parameters())
    bad, checked = [], 0
    for name, p in nat.named_parameters():
        q = rg[name]
        if q.grad is None or q.grad.norm() < 1e-8:
            continue
        assert p.grad is not None, name
        if "word" in name or "position" in name or "token_type" in name:
            rows = q.grad.abs().sum(1) > 0           # only the rows the batch touched
            c = _cos(p.grad[rows], q.grad[rows])
        else:
            c = _cos(p.grad, q.grad)
        checked += 1
        if c < 0.99:
            bad.append((name, round(c, 4)))
    assert checked >= NBLK * 12, checked
    assert not bad, bad


def test_bert_base_width_training_trajectory_tracks_fp32(gpu):
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    m, xs, y = _setup(gpu, seed=3)
    steps, lr = 30, 0.02
    eng = TrainingEngine(copy.deepcopy(m), softmax_cross_entropy, SGD(learningrate=lr, momentum=0.9, dampening=0.0))
    ln = [float(eng.train_step(xs, y).float().item()) for _ in range(steps)]
    ref = copy.deepcopy(m).to(gpu).train()
    opt = torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.9)
    lr_ = []
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(_ref_forward(ref, xs), y)
        loss.backward()
        opt.step()
        lr_.append(loss.item())
    for a, b in zip(ln, lr_):
        assert abs(a - b) < 0.02, (ln, lr_)
    assert ln[-1] < ln[0] - 0.3, ln
