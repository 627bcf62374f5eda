"""Per-generation replay exchange between self-play ranks.

One process per GPU plays its own games; once per generation every rank's finished-game
sample rows are pooled on every rank with ONE padded all-gather (RCCL over xGMI with the
"nccl" backend; gloo on CPU in the tests), replacing the reference's pickle-over-pipe
return of `one_self_play` results to the Trainer (train.py:220-223).  Rows keep the
engine's layout: canonical own/opp bitboards, pi float32[65], TD(lambda) target, player.
The best net's weights travel the other way with `broadcast_state_dict` after a promotion
(train.py:361-367).
"""
import numpy as np
import torch
import torch.distributed as dist

ROW_BYTES = 288  # own u64 | opp u64 | pi f32[65] | z f64 | player i8 | pad (byte rows: bit-exact)


def _t(x, device):
    if isinstance(x, np.ndarray) and x.dtype == np.uint64:
        x = x.view(np.int64)
    return torch.as_tensor(x, device=device)


def pack_rows(s, device):
    """Engine sample dict (numpy or torch) -> uint8 [n, ROW_BYTES] tensor on `device`."""
    own = _t(s["own"], device).to(torch.int64).reshape(-1, 1)
    n = own.shape[0]
    rows = torch.zeros(n, ROW_BYTES, dtype=torch.uint8, device=device)
    if n:
        rows[:, 0:8] = own.view(torch.uint8)
        rows[:, 8:16] = _t(s["opp"], device).to(torch.int64).reshape(-1, 1).view(torch.uint8)
        rows[:, 16:276] = _t(s["pi"], device).to(torch.float32).reshape(n, 65).contiguous() \
            .view(torch.uint8)
        rows[:, 276:284] = _t(s["z"], device).to(torch.float64).reshape(-1, 1).view(torch.uint8)
        rows[:, 284] = _t(s["player"], device).to(torch.int8).view(torch.uint8)
    return rows


def unpack_rows(rows):
    """uint8 [n, ROW_BYTES] -> dict of torch tensors (own/opp int64 bit patterns).  Each
    field is cloned before the dtype view: a 1-row or empty slice counts as contiguous
    and keeps its byte offset, which a wider view rejects."""
    f = lambda a, b: rows[:, a:b].clone()  # noqa: E731
    return {"own": f(0, 8).view(torch.int64).reshape(-1),
            "opp": f(8, 16).view(torch.int64).reshape(-1),
            "pi": f(16, 276).view(torch.float32),
            "z": f(276, 284).view(torch.float64).reshape(-1),
            "player": f(284, 285).view(torch.int8).reshape(-1)}


def allgather_samples(s, device, group=None):
    """Pool every rank's rows on every rank: one all_gather of the counts, one
    all_gather_into_tensor of the rows padded to the largest count."""
    rows = pack_rows(s, device)
    world = dist.get_world_size(group)
    cnt = torch.tensor([rows.shape[0]], dtype=torch.int64, device=device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    mx = max(counts) if counts else 0
    if mx == 0:  # no rank has rows: every rank agrees from the counts, skip the empty collective
        return unpack_rows(rows), counts
    pad = torch.zeros(mx, ROW_BYTES, dtype=torch.uint8, device=device)
    pad[:rows.shape[0]] = rows
    out = torch.empty(world * mx, ROW_BYTES, dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(out, pad, group=group)
    keep = torch.cat([out[r * mx:r * mx + c] for r, c in enumerate(counts)])
    return unpack_rows(keep), counts


def broadcast_state_dict(net, src=0, group=None):
    """Best-net weights from `src` to every rank (after a promotion)."""
    for p in list(net.parameters()) + list(net.buffers()):
        dist.broadcast(p.data, src=src, group=group)
    return net
