"""Linear-chain CRF (the sequence classifier of the reference's NER / intent
models, nlp-architect's CRF behind Py/tfpark/text/keras/ner.py:21-73).

``crf_nll`` is the negative log-likelihood via the forward algorithm (log-space,
one [B, L, L] logsumexp per time step) and ``crf_decode`` the Viterbi path.
``mask`` [B, T] marks real tokens (the reference's 'pad' mode); sequences are
assumed left-aligned. Both run as batched torch ops on the device of the
emissions; the time loop is T small launches (T <= a few hundred).
"""
import torch


def crf_nll(emissions, tags, transitions, mask=None, start=None, end=None):
    """emissions [B, T, L] (float), tags [B, T] (int), transitions [L, L]
    (score of i -> j). Returns the mean negative log-likelihood over the batch."""
    B, T, L = emissions.shape
    e = emissions.float()
    tags = tags.long()
    m = torch.ones(B, T, device=e.device) if mask is None else mask.float()
    tr = transitions.float()
    st = torch.zeros(L, device=e.device) if start is None else start.float()
    en = torch.zeros(L, device=e.device) if end is None else end.float()
    # score of the gold path
    bidx = torch.arange(B, device=e.device)
    gold = st[tags[:, 0]] + e[bidx, 0, tags[:, 0]]
    for t in range(1, T):
        step = tr[tags[:, t - 1], tags[:, t]] + e[bidx, t, tags[:, t]]
        gold = gold + step * m[:, t]
    lengths = m.sum(1).long().clamp_min(1)
    last = tags[bidx, lengths - 1]
    gold = gold + en[last]
    # partition function
    alpha = st.unsqueeze(0) + e[:, 0]                               # [B, L]
    for t in range(1, T):
        nxt = torch.logsumexp(alpha.unsqueeze(2) + tr.unsqueeze(0), dim=1) + e[:, t]
        keep = m[:, t].unsqueeze(1)
        alpha = nxt * keep + alpha * (1 - keep)
    logz = torch.logsumexp(alpha + en.unsqueeze(0), dim=1)
    return (logz - gold).mean()


@torch.no_grad()
def crf_decode(emissions, transitions, mask=None, start=None, end=None):
    """Viterbi decoding -> [B, T] int64 tags (positions past a sequence's length are 0)."""
    B, T, L = emissions.shape
    e = emissions.float()
    m = torch.ones(B, T, device=e.device) if mask is None else mask.float()
    tr = transitions.float()
    st = torch.zeros(L, device=e.device) if start is None else start.float()
    en = torch.zeros(L, device=e.device) if end is None else end.float()
    score = st.unsqueeze(0) + e[:, 0]
    back = []
    for t in range(1, T):
        cand = score.unsqueeze(2) + tr.unsqueeze(0)                 # [B, from, to]
        best, arg = cand.max(dim=1)
        nxt = best + e[:, t]
        keep = m[:, t].unsqueeze(1)
        score = nxt * keep + score * (1 - keep)
        # padded steps point to themselves so backtracking passes through them
        ident = torch.arange(L, device=e.device).unsqueeze(0).expand(B, L)
        back.append(torch.where(keep.bool(), arg, ident))
    score = score + en.unsqueeze(0)
    out = torch.zeros(B, T, dtype=torch.long, device=e.device)
    cur = score.argmax(1)
    out[:, T - 1] = cur
    for t in range(T - 2, -1, -1):
        cur = back[t].gather(1, cur.unsqueeze(1)).squeeze(1)
        out[:, t] = cur
    lengths = m.sum(1).long()
    # realign: tag at the last real position is the argmax state; padded tail zeroed
    pos = torch.arange(T, device=e.device).unsqueeze(0)
    return torch.where(pos < lengths.unsqueeze(1), out, torch.zeros_like(out))
