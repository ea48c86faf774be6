"""INTEGRATION.md's bindings are executed and compiled, not just read.

- The ABI structs' sizeof / offsetof from a C unit compiled against
  include/os_mcts.h equal the ctypes layouts in os_amd/_lib.py and in
  INTEGRATION.md §2's `_Params`, and the library's own os_abi_struct_size.
- INTEGRATION.md §2's ctypes block runs as written (CPU: import + layout
  assert; GPU: `_gpu_search` equals the oracle's numpy-policy MCTSBot,
  mcts.py:346-443).
- §3's C++ bot and §4's C root-parallel snippet compile against the header.
- A params struct whose `reserved` word is not 0 (what a binding built
  against the round-2 9-field struct passes) is refused with OS_ERR_INVALID.
"""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR_DIR = os.path.join(ROOT, "include")
DOC = os.path.join(ROOT, "INTEGRATION.md")
LIB = os.path.join(ROOT, "open_spiel-1_amd", "os_amd", "libos_mcts.so")

STRUCTS = {
    "os_mcts_params": ["uct_c", "max_simulations", "n_rollouts", "max_memory_mb",
                       "solve", "policy", "block_size", "layout", "arena_nodes",
                       "child_selection", "reserved"],
    "os_game_info": ["kind", "num_distinct_actions", "max_game_length", "num_players",
                     "max_children", "rows", "cols", "min_utility", "max_utility",
                     "utility_sum", "komi", "handicap", "state_bytes"],
    "os_selfplay_options": ["temperature", "temperature_drop", "resign", "cutoff_value",
                            "cutoff_probability"],
}


def _code_blocks(lang):
  text = open(DOC).read()
  return re.findall(r"```%s\n(.*?)```" % lang, text, flags=re.S)


def _block(lang, marker):
  hits = [b for b in _code_blocks(lang) if marker in b]
  assert len(hits) == 1, "INTEGRATION.md: expected one %s block with %r" % (lang, marker)
  return hits[0]


@pytest.fixture(scope="module")
def c_layout():
  """{struct: (sizeof, {field: offset})} as gcc lays out include/os_mcts.h."""
  lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "os_mcts.h"',
           'int main(void) {']
  for s, fields in STRUCTS.items():
    lines.append('  printf("%s %%zu\\n", sizeof(%s));' % (s, s))
    for f in fields:
      lines.append('  printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (s, f, s, f))
  lines.append('  return 0; }')
  with tempfile.TemporaryDirectory() as d:
    src, exe = os.path.join(d, "probe.c"), os.path.join(d, "probe")
    open(src, "w").write("\n".join(lines))
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", HDR_DIR, "-o", exe,
                           src])
    out = subprocess.check_output([exe]).decode().split("\n")
  lay = {s: [0, {}] for s in STRUCTS}
  for line in filter(None, out):
    k, v = line.split()
    if "." in k:
      s, f = k.split(".")
      lay[s][1][f] = int(v)
    else:
      lay[k][0] = int(v)
  return lay


def _ctypes_layout(cls):
  return ctypes.sizeof(cls), {f: getattr(cls, f).offset for f, _ in cls._fields_}


def test_product_binding_layout_matches_header(c_layout):
  from os_amd import _lib
  for name, cls in (("os_mcts_params", _lib.MctsParams), ("os_game_info", _lib.GameInfo),
                    ("os_selfplay_options", _lib.SelfPlayOptions)):
    size, offs = _ctypes_layout(cls)
    assert [f for f, _ in cls._fields_] == STRUCTS[name]
    assert size == c_layout[name][0], name
    assert offs == c_layout[name][1], name
    assert _lib.lib.os_abi_struct_size(name.encode()) == size


def test_library_rejects_unknown_struct_name():
  from os_amd import _lib
  assert _lib.lib.os_abi_struct_size(b"os_no_such_struct") == _lib.OS_ERR_INVALID
  assert b"unknown ABI struct" in _lib.lib.os_last_error()


def _exec_section2():
  ns = {}
  os.environ["OS_MCTS_LIB"] = LIB
  exec(compile(_block("python", "class _Params"), "INTEGRATION.md#2", "exec"), ns)
  return ns


def test_section2_ctypes_block_runs_and_matches_header(c_layout):
  ns = _exec_section2()  # includes the block's own os_abi_struct_size assert
  size, offs = _ctypes_layout(ns["_Params"])
  assert [f for f, _ in ns["_Params"]._fields_] == STRUCTS["os_mcts_params"]
  assert (size, offs) == tuple(c_layout["os_mcts_params"])


def _syntax_check(lang, src, extra=()):
  with tempfile.TemporaryDirectory() as d:
    path = os.path.join(d, "snippet." + ("cc" if lang == "c++" else "c"))
    open(path, "w").write(src)
    cc = "g++" if lang == "c++" else "gcc"
    std = "-std=c++17" if lang == "c++" else "-std=c11"
    subprocess.check_call([cc, std, "-fsyntax-only", "-Wall", "-Werror", "-I", HDR_DIR,
                           *extra, path])


# Test-only declarations of the three reference names §3's bot uses, with the
# reference's signatures (spiel.h Game / State, spiel_bots.h Bot,
# spiel_utils.h SpielFatalError); nothing of the reference is compiled.
_SPIEL_DECLS = r"""
#include <cstdint>
#include <random>
#include <sstream>
#include <string>
#include <vector>
namespace open_spiel {
using Action = int64_t;
class Game { public: virtual ~Game() = default; virtual int NumDistinctActions() const = 0;
             virtual std::string ToString() const = 0; };
class State { public: virtual ~State() = default;
              virtual std::vector<Action> History() const = 0; };
class Bot { public: virtual ~Bot() = default; virtual Action Step(const State& state) = 0; };
[[noreturn]] void SpielFatalError(const std::string& error_msg);
}  // namespace open_spiel
using namespace open_spiel;
"""


def test_section3_cpp_bot_compiles():
  src = _block("cpp", "class GpuMCTSBot")
  _syntax_check("c++", _SPIEL_DECLS + src)


def test_section4_c_root_parallel_snippet_compiles():
  body = _block("c", "os_root_parallel")
  _syntax_check("c", '#include "os_mcts.h"\n#include <stddef.h>\nint f(void) {\n' + body +
                "\nreturn 0; }\n", extra=("-Wno-unused-variable",))


@pytest.mark.gpu
def test_section2_gpu_search_equals_oracle(require_gpu):
  import oracle_lib as O
  ns = _exec_section2()
  gs = "connect_four"
  eng = ns["_engine"](gs)
  g = O.Game(gs)
  A = g.num_distinct_actions
  for seed, hist in ((3, []), (11, [3, 3, 2])):
    class Bot:  # the attributes mcts.MCTSBot has (mcts.py:219-262)
      uct_c, max_simulations, solve = 2.0, 300, True
      evaluator = type("E", (), {"n_rollouts": 1})()
      _random_state = np.random.RandomState(seed)

    class St:
      def history(self):
        return hist

      def get_game(self):
        return type("G", (), {"num_distinct_actions": lambda self: A})()

    out, one = ns["_gpu_search"](eng, St(), Bot)
    ref = g.mcts_numpy(hist, seed, uct_c=2.0, max_simulations=300)
    nc = ref["nchild"][0]
    assert one[0][0] == nc
    for got, k in zip(out, ("child_action", "child_n", "child_w", "child_out")):
      np.testing.assert_array_equal(got[:nc], ref[k][0][:nc])
    assert one[1][0] == ref["root_n"][0] and one[2][0] == ref["root_w"][0]
    assert one[4][0] == ref["best_action"][0]
    # the shared RandomState continues exactly where the reference's would
    assert Bot._random_state.randint(0, 2**32, dtype=np.uint32) == ref["next_word"][0]


@pytest.mark.gpu
def test_nonzero_reserved_is_refused(require_gpu):
  from os_amd import _lib
  from os_amd import engine as E
  eng = E.Engine("tic_tac_toe", device=0)
  p = _lib.MctsParams(2.0, 10, 1, 1000, 1, 0, 0, 2, 0, 0, 7)
  acts, offs = np.zeros(0, np.int64), np.zeros(2, np.int64)
  seeds = np.zeros(1, np.uint32)
  rc = _lib.lib.os_engine_prepare(eng._h, ctypes.byref(p), 1, _lib.ptr(acts),
                                  _lib.ptr(offs), _lib.ptr(seeds), _lib.ptr(seeds))
  assert rc == _lib.OS_ERR_INVALID
  assert b"reserved" in _lib.lib.os_last_error()
