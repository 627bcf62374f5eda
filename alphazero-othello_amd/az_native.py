"""ctypes binding of the C-ABI library `libaz_othello.so` (include/az_othello.h).

The whole product path goes through this module: the OthelloGameNew drop-in
(envs/othello.py), the MCTS drop-in (MCTS_model.py) and the batched self-play engine
(engine.py).  There is no fallback: if the library is missing this module raises on
import, naming the build command.

Error mapping follows the reference's Python conventions:
AZ_ERR_ILLEGAL -> ValueError("Illegal move: a") (envs/othello.py:421),
AZ_ERR_STATE -> KeyError(action) (MCTS_model.py:214), everything else -> RuntimeError.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# AZ_LIB_PATH: an alternative build of the same library (experiment builds, scripts/exp)
LIB_PATH = os.environ.get("AZ_LIB_PATH") or os.path.join(HERE, "libaz_othello.so")

AZ_OK = 0
AZ_ERR_ILLEGAL = -1
AZ_ERR_ARG = -2
AZ_ERR_HIP = -3
AZ_ERR_CAPACITY = -4
AZ_ERR_STATE = -5

AZ_FLAG_TERMINAL = 1
AZ_FLAG_NOPLACE = 2
AZ_FLAG_ILLEGAL = 4
AZ_FLAG_PASSED = 8

AZ_EVAL_EXTERNAL, AZ_EVAL_ROLLOUT = 0, 1
AZ_RNG_DEVICE, AZ_RNG_INJECTED = 0, 1
AZ_GAME_IDLE, AZ_GAME_ACTIVE, AZ_GAME_FINISHED, AZ_GAME_SEARCH_DONE = 0, 1, 2, 3


class AzConfig(ctypes.Structure):
    _fields_ = [
        ("n_games", ctypes.c_int32),
        ("node_capacity", ctypes.c_int32),
        ("max_plies", ctypes.c_int32),
        ("num_simulations", ctypes.c_int32),
        ("c_puct", ctypes.c_double),
        ("dirichlet_alpha", ctypes.c_double),
        ("dirichlet_epsilon", ctypes.c_double),
        ("temperature", ctypes.c_double),
        ("num_exploratory_moves", ctypes.c_int32),
        ("lambd", ctypes.c_double),
        ("eval_mode", ctypes.c_int32),
        ("rng_mode", ctypes.c_int32),
        ("d4_augment", ctypes.c_int32),
        ("auto_play", ctypes.c_int32),
        ("refill", ctypes.c_int32),
        ("sample_capacity", ctypes.c_int64),
        ("inj_noise_slots", ctypes.c_int32),
        ("inj_uniform_slots", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("stream_id", ctypes.c_uint64),
        ("leaves_per_step", ctypes.c_int32),
    ]


_P = ctypes.c_void_p
_I = ctypes.c_int
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_D = ctypes.c_double

AZ_CONV_SPLIT3, AZ_CONV_FP16, AZ_CONV_FP16X2 = 0, 1, 2  # conv kernel numerics modes

# name -> argtypes (restype is int for every entry point except az_last_error)
SIGNATURES = {
    "az_abi_version": [],
    "oth_legal_cpu": [_P, _P, _P, _I64],
    "oth_step_cpu": [_P, _P, _P, _P, _P, _P, _P, _I64],
    "oth_make_move_cpu": [_P, _P, _P, _P, _P, _I64],
    "oth_pack_np": [_P, _P, _P, _P, _I64],
    "oth_unpack_np": [_P, _P, _P, _P, _I64],
    "oth_d4_cpu": [_P, _P, _P, _I64],
    "oth_legal_gpu": [_P, _P, _P, _I64, _P],
    "oth_step_gpu": [_P, _P, _P, _P, _P, _P, _P, _I64, _P],
    "oth_d4_gpu": [_P, _P, _P, _I64, _P],
    "oth_step_io_gpu": [_P, _P, _P, _P, _P, _P, _P, _I64, _P],
    "az_engine_create": [ctypes.POINTER(AzConfig), ctypes.POINTER(_P)],
    "az_engine_destroy": [_P],
    "az_engine_geometry": [_P, _P, _P, _P],
    "az_reset_all": [_P, _I64, _I32, _P],
    "az_set_root": [_P, _I32, _U64, _U64, _I32, _P],
    "az_begin_search": [_P, _I32, _I32, _P],
    "az_select": [_P, _P, _P, _P],
    "az_expand_backup": [_P, _P, _P, _P],
    "az_play": [_P, _P],
    "az_engine_defer_moves": [_P, _I32],
    "az_engine_set_stem": [_P, _P, _P, _P, _P, _I32],
    "az_select_move": [_P, _P, _P, _I32, _P],
    "az_select_move_expand": [_P, _P, _P, _P, _P, _I32, _P],
    "az_select_expand": [_P, _P, _P, _P, _P, _P],
    "az_expand_backup_par": [_P, _P, _P, _I32, _P],
    "az_move_flush": [_P, _I32, _P],
    "az_inject": [_P, _P, _P, _P],
    "az_root_policy": [_P, _I32, _D, _D, _P, _P, _P, _P],
    "az_make_move": [_P, _I32, _I32, _P],
    "az_counters": [_P, _P, _P],
    "az_set_roots": [_P, _P, _P, _P, _P, _I32, _P],
    "az_begin_search_slots": [_P, _P, _I32, _I32, _P],
    "az_root_stats": [_P, _P, _P, _P],
    "az_reroot_slots": [_P, _P, _P, _P],
    "az_game_info": [_P, _P, _P, _P, _P, _P, _P, _P],
    "az_export_tree": [_P, _I32, _I32] + [_P] * 14,
    "az_export_trajectory": [_P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P],
    "az_samples": [_P, _P, _P, _P, _P, _P, _P, _P],
    "az_copy_samples": [_P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P],
    "az_clear_samples": [_P, _P],
    "az_bias_act_gpu": [_P, _P, _P, _I64, _I32, _I32, _P],
    "az_conv3x3_gpu": [_P, _P, _P, _P, _P, _I32, _I32, _I32, _P],
    "az_conv_stem_gpu": [_P, _P, _P, _P, _I32, _I32, _P],
    "az_conv_stem2_gpu": [_P, _P, _P, _P, _I32, _I32, _P, _P],
    "az_conv3x3_cfg_gpu": [_P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _P],
    "az_conv3x3_mx_prep_gpu": [_P, _P, _I32, _I32, _P],
    "az_conv3x3_mx_prep_bytes": [_I32, _I32],
    "az_heads_fast_gemm_gpu": [_P, _P, _P, _I32, _P, _I32, _I32, _I32, _I32, _P],
    "az_fast_trunk_gpu": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P],
    "az_conv3x3_mx_gpu": [_P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _P],
    "az_conv3x3_wino_prep_gpu": [_P, _P, _I32, _I32, _P],
    "az_conv3x3_wino_gpu": [_P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _P],
    "az_conv3x3_wino4_gpu": [_P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _P, _P, _P],
    "az_conv3x3_wino4_splitk_gpu": [_P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _P, _P, _P,
                                    _I32, _P],
    "az_conv3x3_wino4_heads_gpu": [_P, _P, _P, _P, _I32, _I32, _I32] + [_P] * 11 + [_P],
    "az_board_absmax_gpu": [_P, _I32, _I32, _P, _P],
    "az_conv3x3_wino_prep_bytes": [_I32, _I32],
    "az_trunk_wino_gpu": [_P] * 7 + [_I32] * 4 + [_P],
    "az_trunk_wino4_gpu": [_P] * 11 + [_I32] * 3 + [_P],
    "az_trunk_wino4_heads_gpu": [_P] * 11 + [_I32] * 3 + [_P] * 10 + [_P],
    "az_trunk_wino4_heads_fp16_gpu": [_P] * 11 + [_I32] * 3 + [_P] * 10 + [_P],
    "az_heads_az_gpu": [_P] * 11 + [_I32, _I32, _P],
    "az_heads_fast_finish_gpu": [_P, _I32, _I32, _P, _P, _P, _P, _P, _I32, _P],
    "az_conv3x3_mx_cfg_gpu": [_P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _P],
    "az_conv3x3_mx_stem_gpu": [_P] * 7 + [_I32, _I32, _I32, _I32, _P],
    "az_replay_aggregate_gpu": [_P] * 5 + [_I64] + [_P] * 10,
}


def _load():
    # torch ships its own HIP runtime and preloads it by path; loading ours first would put
    # a second copy of libamdhip64 / libhsa-runtime64 in the process (the second HSA
    # instance then sees no device).  With torch loaded first, the library's
    # libamdhip64.so.7 dependency resolves to torch's copy by soname: one runtime.
    import torch  # noqa: F401

    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python __graft_entry__.py` (build()) "
            "or `python alphazero-othello_amd/az_build.py`; there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name in ("az_last_error", "az_build_id"):
        getattr(lib, name).argtypes = []
        getattr(lib, name).restype = ctypes.c_char_p
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _I
    lib.az_conv3x3_wino_prep_bytes.restype = _I64
    lib.az_conv3x3_mx_prep_bytes.restype = _I64
    return lib


lib = _load()


def build_id():
    """sha256 of the sources the loaded library was compiled from (az_build.source_hash)."""
    return lib.az_build_id().decode()


def last_error():
    m = lib.az_last_error()
    return m.decode() if m else ""


def check(rc, what=""):
    """Raise the reference's exception type for a failed C-ABI call."""
    if rc == AZ_OK:
        return
    msg = last_error()
    if rc == AZ_ERR_ILLEGAL:
        raise ValueError(msg or f"Illegal move ({what})")
    if rc == AZ_ERR_STATE:
        try:
            key = int(msg.split(":")[0])
        except ValueError:
            key = msg
        raise KeyError(key)
    raise RuntimeError(f"{what} failed ({rc}): {msg}")


def ptr(a):
    """Host numpy array or device torch tensor -> void*."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"], "buffer must be C-contiguous"
        return a.ctypes.data_as(_P)
    return _P(a.data_ptr())  # torch tensor


def stream_ptr(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return _P(s.cuda_stream)


# ---- thin typed wrappers over the stateless CPU board entry points ----------------------

def _u64(x):
    return np.ascontiguousarray(x, dtype=np.uint64)


def legal_cpu(own, opp):
    own, opp = _u64(own), _u64(opp)
    out = np.empty(own.shape, np.uint64)
    check(lib.oth_legal_cpu(ptr(own), ptr(opp), ptr(out), own.size), "oth_legal_cpu")
    return out


def step_cpu(own, opp, act, raise_illegal=True):
    own, opp = _u64(own), _u64(opp)
    act = np.ascontiguousarray(act, dtype=np.uint8)
    n = own.size
    o, p, lg = (np.empty(own.shape, np.uint64) for _ in range(3))
    st = np.empty(own.shape, np.uint16)
    rc = lib.oth_step_cpu(ptr(own), ptr(opp), ptr(act), ptr(o), ptr(p), ptr(lg), ptr(st), n)
    if rc != AZ_OK and (raise_illegal or rc != AZ_ERR_ILLEGAL):
        check(rc, "oth_step_cpu")
    return o, p, lg, st


def make_move_cpu(own, opp, act):
    own, opp = _u64(own), _u64(opp)
    act = np.ascontiguousarray(act, dtype=np.uint8)
    o, p = np.empty(own.shape, np.uint64), np.empty(own.shape, np.uint64)
    check(lib.oth_make_move_cpu(ptr(own), ptr(opp), ptr(act), ptr(o), ptr(p), own.size),
          "oth_make_move_cpu")
    return o, p


def pack_np(states, player):
    states = np.ascontiguousarray(states, dtype=np.int8).reshape(-1, 64)
    player = np.ascontiguousarray(np.broadcast_to(player, (states.shape[0],)), dtype=np.int8)
    n = states.shape[0]
    own, opp = np.empty(n, np.uint64), np.empty(n, np.uint64)
    check(lib.oth_pack_np(ptr(states), ptr(player), ptr(own), ptr(opp), n), "oth_pack_np")
    return own, opp


def unpack_np(own, opp, player):
    own, opp = _u64(own).reshape(-1), _u64(opp).reshape(-1)
    n = own.size
    player = np.ascontiguousarray(np.broadcast_to(player, (n,)), dtype=np.int8)
    out = np.empty((n, 64), np.int8)
    check(lib.oth_unpack_np(ptr(own), ptr(opp), ptr(player), ptr(out), n), "oth_unpack_np")
    return out.reshape(n, 8, 8)


def d4_cpu(x, sym):
    x = _u64(x)
    sym = np.ascontiguousarray(np.broadcast_to(sym, x.shape), dtype=np.uint8)
    out = np.empty(x.shape, np.uint64)
    check(lib.oth_d4_cpu(ptr(x), ptr(sym), ptr(out), x.size), "oth_d4_cpu")
    return out


def status_flags(st):
    return np.asarray(st) & 0xFF


def status_score(st):
    return (np.asarray(st) >> 8).astype(np.uint8).view(np.int8).astype(np.int32)
