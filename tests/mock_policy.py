"""Deterministic mock policy/value function used by every MCTS parity test.

The reference nets (Models.py) are random-init here (no checkpoints offline), so MCTS
parity is pinned with a closed-form policy instead.  The function is
integer arithmetic on the canonical board x = player*state (Models.py:16), so numpy, the
reference MCTS and the GPU engine's evaluator produce bit-identical priors and values:

    h_a     = 1 + ((A @ (x+1))_a mod 1021)       a in 0..64
    prior_a = float32(h_a) / 1024                 (exact in float32, NOT normalised:
                                                   the MCTS masks and renormalises)
    value   = (((B @ (x+1)) mod 2001) - 1000) / 1024   (exact in float32)
"""
import numpy as np

_i = np.arange(65, dtype=np.int64)[:, None]
_j = np.arange(64, dtype=np.int64)[None, :]
A = ((_i * 131 + _j * 71 + _i * _j * 7) % 97).astype(np.int64)  # [65, 64]
B = ((np.arange(64, dtype=np.int64) * 37 + 11) % 89).astype(np.int64)  # [64]


def _mats(salt):
    """salt 0 = the golden-vector policy; other salts = distinct "nets" (arena tests)."""
    if salt == 0:
        return A, B
    a = ((_i * 131 + _j * 71 + _i * _j * 7 + 13 * salt) % 97).astype(np.int64)
    b = ((np.arange(64, dtype=np.int64) * 37 + 11 + 5 * salt) % 89).astype(np.int64)
    return a, b


def mock_eval(canonical, salt=0):
    """canonical: int array [..., 64] with values in {-1, 0, +1}.
    Returns priors float32 [..., 65] and values float64 [...] (float32-exact)."""
    A, B = _mats(salt)
    x = np.asarray(canonical).astype(np.int64) + 1
    h = (x @ A.T) % 1021 + 1
    priors = h.astype(np.float32) / np.float32(1024)
    k = (x @ B) % 2001
    values = (k - 1000) / 1024.0
    return priors, values


class MockPolicy:
    """Duck-typed `policy` for the reference MCTS (policy.inference(state, player))."""

    def inference(self, state, current_player):
        canon = (current_player * np.asarray(state)).reshape(-1)
        p, v = mock_eval(canon)
        return p.astype(np.float32), float(v)


class MockPolicyNet(MockPolicy):
    """Constructible the way one_self_play builds its net (self_play_worker.py:43-46)."""

    def __init__(self, **cfg):
        pass

    def load_state_dict(self, sd):
        return None

    def eval(self):
        return self

    def get_config(self):
        return {}


def mock_eval_planes(nn_in):
    """Evaluator for the engine: nn_in float [B, 64] canonical planes (+1/-1/0)."""
    x = np.rint(np.asarray(nn_in, np.float32)).astype(np.int64).reshape(-1, 64)
    p, v = mock_eval(x)
    return p, v.astype(np.float32)


def mock_eval_torch(planes, salt=0):
    """The same closed form on device (torch float64 matmuls are exact here: every partial
    sum is an integer below 2^53).  planes: float32 [G, 64] -> (priors f32 [G, 65],
    values f32 [G])."""
    import torch

    A, B = _mats(salt)
    x = torch.round(planes.double()) + 1.0
    At = torch.as_tensor(A.T, dtype=torch.float64, device=planes.device)
    Bt = torch.as_tensor(B, dtype=torch.float64, device=planes.device)
    h = torch.remainder(x @ At, 1021.0) + 1.0
    k = torch.remainder(x @ Bt, 2001.0)
    return (h / 1024.0).float().contiguous(), ((k - 1000.0) / 1024.0).float().contiguous()


def MockNet(salt=0):
    """The mock policy (salt: mock_eval's distinct "nets") as a module BatchedSelfPlay evaluates (fold=False, evaluate_planes), its
    matrices resident on the device so the step is graph-capturable (mock_eval_torch's closed
    form, exact in float64)."""
    import torch

    class _MockNet(torch.nn.Module):
        def __init__(self):
            super().__init__()
            A, B = _mats(salt)
            self.register_buffer("At", torch.as_tensor(A.T, dtype=torch.float64))
            self.register_buffer("Bt", torch.as_tensor(B, dtype=torch.float64))

        def evaluate_planes(self, planes):
            x = torch.round(planes.double()) + 1.0
            h = torch.remainder(x @ self.At, 1021.0) + 1.0
            k = torch.remainder(x @ self.Bt, 2001.0)
            return ((h / 1024.0).float().contiguous(),
                    ((k - 1000.0) / 1024.0).float().contiguous())

        def evaluate_into(self, planes, priors, values):
            p, v = self.evaluate_planes(planes)
            priors.copy_(p)
            values.copy_(v)

    return _MockNet()
