"""ctypes binding of libos_mcts.so (the C-ABI declared in include/os_mcts.h).

The library is built in-tree by `__graft_entry__.build()` (hipcc, gfx950).
Loading it is mandatory: there is no Python or CPU fallback for the search
path — if the .so is missing this module raises ImportError.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# OS_AMD_LIB selects another build of the same library (A/B kernel variants).
LIB_PATH = os.environ.get("OS_AMD_LIB") or os.path.join(_HERE, "libos_mcts.so")

OS_OK = 0
OS_ERR_INVALID = -1
OS_ERR_UNSUPPORTED = -2
OS_ERR_DEVICE = -3
OS_ERR_CAPACITY = -4

POLICY_CPP = 0
POLICY_NUMPY = 1

SELECT_UCT = 0
SELECT_PUCT = 1

LAYOUT_WAVE = 0
LAYOUT_LANE = 1
LAYOUT_AUTO = 2

if not os.path.exists(LIB_PATH):
  raise ImportError(
      "libos_mcts.so not found at %s: run `python -c \"import __graft_entry__ as g;"
      " g.build()\"` to compile the HIP engine (no CPU fallback exists)" % LIB_PATH)

def _share_torch_hip_runtime():
  """Makes libos_mcts.so bind to the HIP/HSA runtime PyTorch ships, if any.

  A process must hold ONE HIP runtime: PyTorch-ROCm bundles its own
  libamdhip64 / libhsa-runtime64 (same SONAMEs as /opt/rocm's), and a second
  copy loaded beside it cannot open the device.  Preloading torch's copies
  RTLD_GLOBAL (without importing torch) lets the dynamic loader resolve our
  NEEDED entries by SONAME to them, whichever of torch / os_amd is imported
  first.  Set OS_AMD_HIP_RUNTIME=system to skip (processes without torch).
  """
  if os.environ.get("OS_AMD_HIP_RUNTIME", "torch") == "system":
    return
  import importlib.util
  spec = importlib.util.find_spec("torch")
  if spec is None or not spec.submodule_search_locations:
    return
  tlib = os.path.join(list(spec.submodule_search_locations)[0], "lib")
  for name in ("libhsa-runtime64.so", "libamdhip64.so"):
    p = os.path.join(tlib, name)
    if os.path.exists(p):
      ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)


_share_torch_hip_runtime()
lib = ctypes.CDLL(LIB_PATH)

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_dbl = ctypes.c_double
_cp = ctypes.c_char_p


class GameInfo(ctypes.Structure):
  _fields_ = [("kind", _i32), ("num_distinct_actions", _i32),
              ("max_game_length", _i32), ("num_players", _i32),
              ("max_children", _i32), ("rows", _i32), ("cols", _i32),
              ("min_utility", _dbl), ("max_utility", _dbl),
              ("utility_sum", _dbl), ("komi", _dbl), ("handicap", _i32),
              ("state_bytes", _i32)]


class MctsParams(ctypes.Structure):
  _fields_ = [("uct_c", _dbl), ("max_simulations", _i32), ("n_rollouts", _i32),
              ("max_memory_mb", _i64), ("solve", _i32), ("policy", _i32),
              ("block_size", _i32), ("layout", _i32), ("arena_nodes", _i64),
              ("child_selection", _i32), ("reserved", _i32)]


def _sig(name, restype, argtypes):
  f = getattr(lib, name)
  f.restype = restype
  f.argtypes = argtypes
  return f


_P = _vp  # pointers passed as raw addresses (numpy .ctypes.data)

_sig("os_last_error", _cp, [])
_sig("os_build_info", _cp, [])
_sig("os_abi_struct_size", _i64, [_cp])
_sig("os_debug_phase_cycles", ctypes.c_int, [_P, _i32])
_sig("os_game_load", ctypes.c_int, [_cp, ctypes.POINTER(_vp)])
_sig("os_game_free", None, [_vp])
_sig("os_game_get_info", ctypes.c_int, [_vp, ctypes.POINTER(GameInfo)])
_sig("os_game_to_string", _i64, [_vp, _cp, _i64])
_sig("os_state_new", ctypes.c_int, [_vp, ctypes.POINTER(_vp)])
_sig("os_state_clone", ctypes.c_int, [_vp, ctypes.POINTER(_vp)])
_sig("os_state_free", None, [_vp])
_sig("os_state_apply", ctypes.c_int, [_vp, _i64])
_sig("os_state_current_player", _i32, [_vp])
_sig("os_state_is_terminal", _i32, [_vp])
_sig("os_state_returns", ctypes.c_int, [_vp, _P])
_sig("os_state_legal_actions", _i32, [_vp, _P, _i32])
_sig("os_state_history", _i32, [_vp, _P, _i32])
_sig("os_state_to_string", _i64, [_vp, _cp, _i64])
_sig("os_state_action_to_string", _i64, [_vp, _i32, _i64, _cp, _i64])
_sig("os_game_observation_shape", _i64, [_vp, _P])
_sig("os_state_observation_tensor", _i64, [_vp, _i32, _P, _i64])
_sig("os_engine_create", ctypes.c_int, [_cp, _i32, ctypes.POINTER(_vp)])
_sig("os_engine_destroy", ctypes.c_int, [_vp])
_sig("os_mcts_batch", ctypes.c_int,
     [_vp, ctypes.POINTER(MctsParams), _i64, _P, _P, _P, _P, _i32, _P, _P, _P, _P,
      _P, _P, _P, _P, _P, _P])
_sig("os_mcts_stateful", ctypes.c_int,
     [_vp, ctypes.POINTER(MctsParams), _P, _i64, _i32, _P, _P, _P, _P, _i32, _P,
      _P, _P, _P, _P, _P, _P, _P, _P, _P])
_sig("os_engine_tree", ctypes.c_int, [_vp, _i64, _P, _P, _P, _P, _P, _P, _P])
_sig("os_rollouts_batch", ctypes.c_int, [_vp, _P, _i64, _i64, _i32, _P, _P])
_sig("os_engine_prepare", ctypes.c_int,
     [_vp, ctypes.POINTER(MctsParams), _i64, _P, _P, _P, _P])
_sig("os_engine_run_async", ctypes.c_int, [_vp, _vp])
_sig("os_engine_fetch", ctypes.c_int,
     [_vp, _i32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P])
_sig("os_engine_last_sims", _i64, [_vp])
_sig("os_engine_stats", ctypes.c_int, [_vp, _P])
_sig("os_engine_set_arena_mode", ctypes.c_int, [_vp, ctypes.c_int32])
_sig("os_engine_arena_info", ctypes.c_int, [_vp, _P])
_sig("os_engine_set_rollout_layout", ctypes.c_int, [_vp, _i32])
_sig("os_rollouts_prepare", ctypes.c_int, [_vp, _P, _i64, _i64, _i32, _P])
_sig("os_rollouts_run_async", ctypes.c_int, [_vp, _vp])
_sig("os_rollouts_fetch", ctypes.c_int, [_vp, _P])
_sig("os_rollouts_outcomes_async", ctypes.c_int, [_vp, _vp, _vp])
_sig("os_rollouts_stats", ctypes.c_int, [_vp, _vp])
_sig("os_engine_root_sums_async", ctypes.c_int, [_vp, _i32, _vp, _vp, _vp])
_sig("os_state_is_chance_node", _i32, [_vp])
_sig("os_state_chance_outcomes", _i32, [_vp, _P, _P, _i32])
_sig("os_root_parallel", ctypes.c_int,
     [_P, _i32, ctypes.POINTER(MctsParams), _P, _i64, _i64, _u32, _i32, _P, _P, _P])
_sig("os_selfplay", ctypes.c_int,
     [_vp, ctypes.POINTER(MctsParams), _i64, _P, _P, _P, _P, _i32, _P, _P, _P, _P, _P])
_sig("os_selfplay_prepare", ctypes.c_int,
     [_vp, ctypes.POINTER(MctsParams), _i64, _P, _P, _P, _P, _i32, _i32])
_sig("os_selfplay_run_async", ctypes.c_int, [_vp, _vp])
_sig("os_selfplay_fetch", ctypes.c_int, [_vp, _P, _P, _P, _P, _P])
RECORD_VISITS = 1
RECORD_OBSERVATIONS = 2
RECORD_POLICY = 4
RECORD_ROOT_VALUES = 8


class SelfPlayOptions(ctypes.Structure):
  _fields_ = [("temperature", _dbl), ("temperature_drop", _i32), ("resign", _i32),
              ("cutoff_value", _dbl), ("cutoff_probability", _dbl)]


_sig("os_selfplay_set_options", ctypes.c_int,
     [_vp, ctypes.POINTER(SelfPlayOptions), _i64, _P])
_sig("os_selfplay_fetch_targets", ctypes.c_int, [_vp, _P, _P])
_sig("os_az_prepare", ctypes.c_int,
     [_vp, ctypes.POINTER(MctsParams), _i32, _i64, _P, _P, _P, ctypes.c_double,
      ctypes.c_double, _vp, _vp, _vp, _vp, _vp, _vp])
_sig("os_dirichlet_noise", _i64, [_u32, _i32, ctypes.c_double, _P])
_sig("os_az_prepare_stateful", ctypes.c_int,
     [_vp, ctypes.POINTER(MctsParams), _i32, _i64, _P, _P, _P, _P, ctypes.c_double,
      ctypes.c_double, _vp, _vp, _vp, _vp, _vp, _vp])
_sig("os_az_export_rng", ctypes.c_int, [_vp, _P, _P])
_sig("os_az_step_async", ctypes.c_int, [_vp, _vp])
_sig("os_az_heads_async", ctypes.c_int, [_vp, _i32, _i64, _i32, _i64, _vp, _vp, _vp, _vp])
_sig("os_az_mlp_heads_async", ctypes.c_int,
     [_vp, _i64, _i32, _vp, _i32, _vp, _i32, _vp, _vp, _vp, _vp])
_sig("os_az_set_requests", ctypes.c_int, [_vp, ctypes.c_int32])
_sig("os_az_set_layout", ctypes.c_int, [_vp, ctypes.c_int32])
_sig("os_az_get_layout", ctypes.c_int, [_vp, _P])
_sig("os_engine_get_layout", ctypes.c_int, [_vp, _P])
_sig("os_engine_get_searches_per_wave", ctypes.c_int, [_vp, _P])
_sig("os_az_requests", ctypes.c_int, [_vp, _P])
_sig("os_engine_set_run_timing", ctypes.c_int, [_vp, ctypes.c_int32])
_sig("os_engine_last_run_ms", ctypes.c_int, [_vp, _P])
_sig("os_az_stage", ctypes.c_int, [_vp, ctypes.POINTER(MctsParams), _i32, _i64, _P, _P, _P,
                                   ctypes.c_double, ctypes.c_double])
_sig("os_az_prepare_staged", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp])
_sig("os_az_set_noise", ctypes.c_int, [_vp, _P, _i64, ctypes.c_double])
_sig("os_az_tree_priors", ctypes.c_int, [_vp, _i64, _i64, _P])
AZ_REQUESTS_SEPARATE, AZ_REQUESTS_FUSED = 0, 1
_sig("os_az_fetch", ctypes.c_int, [_vp, _i32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P])
_sig("os_engine_node_bytes", _i32, [_vp])
_sig("os_engine_state_bytes", _i32, [_vp])
_sig("os_make_roots", _i64, [_vp, _i64, _u32, _i32, _P, _P])
_sig("os_sample_action", _i32, [_P, _i32, _P, _P])


def _check_abi_layout():
  """The library reports the struct sizes it was built with: a stale build or
  binding fails at import instead of misreading parameters."""
  for name, cls in (("os_mcts_params", MctsParams), ("os_game_info", GameInfo),
                    ("os_selfplay_options", SelfPlayOptions)):
    n = lib.os_abi_struct_size(name.encode())
    if n != ctypes.sizeof(cls):
      raise ImportError("%s: libos_mcts.so has %d bytes, the ctypes binding %d "
                        "(rebuild the library)" % (name, n, ctypes.sizeof(cls)))


_check_abi_layout()


class SpielError(RuntimeError):
  """Raised where the reference raises SpielFatalError (pyspiel RuntimeError)."""


def check(rc):
  """Maps a C-ABI return code to the reference's Python exception types."""
  if rc == OS_OK:
    return
  msg = lib.os_last_error().decode(errors="replace")
  if rc == OS_ERR_UNSUPPORTED:
    raise ValueError(msg)
  raise SpielError(msg)


def ptr(a):
  """Raw data pointer of a C-contiguous numpy array (None -> NULL)."""
  if a is None:
    return None
  assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
  return a.ctypes.data


def get_string(fn, *args):
  n = fn(*args, None, 0)
  buf = ctypes.create_string_buffer(int(n) + 1)
  fn(*args, buf, n + 1)
  return buf.value.decode()


def i64(x):
  return np.ascontiguousarray(x, dtype=np.int64)


def u32(x):
  return np.ascontiguousarray(x, dtype=np.uint32)
