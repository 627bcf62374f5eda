"""Generate tests/golden/net_outputs.npz by running the REFERENCE's nets (Models.py).

Runs only in the build container, where the reference tree is mounted read-only at
/root/reference; the GPU box reads only the committed .npz.

    python tests/golden/make_net_goldens.py

For each of AlphaZeroNet(8, 65, 5, 128) (reference Models.py:164-221, configs[2]'s net) and
FastOthelloNet(8, 65) (Models.py:93-161, configs[1]'s net):
  * build it from the reference module after torch.manual_seed(seed), give every BatchNorm
    random running statistics and affine parameters (so BN folding is exercised), eval();
  * store every state_dict tensor (`<net>/sd/<key>`) -- the test loads them with
    load_state_dict(strict=True) into this repo's Models.py;
  * run the reference forward (fp32, torch CPU) on 1,024 canonical boards drawn from
    board_corpus.npz (player * state, the reference's canonical input, Models.py:16) and store
    softmax(logits) and tanh value;
  * run the reference's batch-1 `Inference.inference(state, player)` (Models.py:9-31) on a
    few absolute-colour states with both players and store (policy, value).
"""
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)


def boards_from_bits(pos, neg):
    """Absolute-colour int8 [n, 8, 8] from the corpus' row-major bitboards (bit r*8+c)."""
    bits = np.arange(64, dtype=np.uint64)
    p = ((pos[:, None] >> bits) & np.uint64(1)).astype(np.int8)
    n = ((neg[:, None] >> bits) & np.uint64(1)).astype(np.int8)
    return (p - n).reshape(-1, 8, 8)


def randomise_bn(net, g):
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.copy_(torch.rand(m.running_mean.shape, generator=g) - 0.5)
            m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) * 1.5 + 0.5)
            m.weight.data.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
            m.bias.data.copy_(torch.rand(m.bias.shape, generator=g) * 0.4 - 0.2)


def main():
    import Models as RM  # the reference's Models.py

    torch.set_num_threads(1)
    corpus = np.load(os.path.join(HERE, "board_corpus.npz"), allow_pickle=False)
    rng = np.random.default_rng(20251018)
    n = len(corpus["pos"])
    idx = np.sort(rng.choice(n, 1024, replace=False))
    states = boards_from_bits(corpus["pos"][idx], corpus["neg"][idx])
    players = corpus["player"][idx].astype(np.int8)
    canon = (states * players[:, None, None]).astype(np.int8)  # Models.py:16
    # batch-1 Inference.inference cases: absolute states with BOTH players
    inf_idx = np.arange(0, 1024, 128)
    inf_states = np.repeat(states[inf_idx], 2, axis=0)
    inf_players = np.tile(np.array([1, -1], np.int8), len(inf_idx))

    out = {"canon": canon, "corpus_index": idx.astype(np.int64),
           "inf_states": inf_states, "inf_players": inf_players}
    for name, make, seed in (("az", lambda: RM.AlphaZeroNet(8, 65, 5, 128), 5),
                             ("fast", lambda: RM.FastOthelloNet(8, 65), 6)):
        torch.manual_seed(seed)
        net = make()
        randomise_bn(net, torch.Generator().manual_seed(seed + 100))
        net.eval()
        for k, v in net.state_dict().items():
            out[f"{name}/sd/{k}"] = v.detach().cpu().numpy()
        with torch.no_grad():
            x = torch.from_numpy(canon.astype(np.float32)).unsqueeze(1)
            logits, val = net(x)
            out[f"{name}/priors"] = torch.softmax(logits, -1).numpy().astype(np.float32)
            out[f"{name}/values"] = val.reshape(-1).numpy().astype(np.float32)
        pol, vals = [], []
        for s, p in zip(inf_states, inf_players):
            pi, v = net.inference(s, int(p))
            pol.append(np.asarray(pi, np.float32))
            vals.append(v)
        out[f"{name}/inf_policy"] = np.stack(pol)
        out[f"{name}/inf_value"] = np.asarray(vals, np.float64)
        print(name, "params", sum(v.numel() for v in net.parameters()),
              "value range", float(val.min()), float(val.max()), flush=True)
    path = os.path.join(HERE, "net_outputs.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
