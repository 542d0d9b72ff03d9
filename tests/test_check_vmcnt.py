"""tools/check_vmcnt.py, the build-time proof of k_rdx's publish waits (kernels_xcd.hip).

The Makefile refuses to link libfmcw when a publish (a no-return agent-scope
``global_atomic_add``) can be reached on some control-flow path with a hand-off slot
store (a ``buffer_store`` without a cache-policy flag) that no ``s_waitcnt vmcnt(N)``
on the way has covered.  These CPU tests feed it hand-written gfx950 assembly: a
covered store, a count one too loose, a branch that skips the wait, and the RD-style
stores (with a cache policy) that are not slot stores; then the code the Makefile
built, when it is there.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_vmcnt as cv  # noqa: E402

HEAD = "_ZN4fmcw5k_rdxILb1ELb0ELb1EEEvNS_11OnePassArgsE:\n"
TAIL = ".Lfunc_end0:\n"


def _run(body: str) -> bool:
    fns = cv.functions(HEAD + body + TAIL, r"k_rdx")
    assert len(fns) == 1
    (name, lines), = fns.items()
    return bool(cv.check_function(name, lines, quiet=True))


def test_covered_store_passes():
    # two vector-memory ops issued after the slot store: vmcnt(2) means it has completed
    assert _run("""
    buffer_store_dwordx4 v[0:3], v4, s[0:3], 0 offen
    global_load_dwordx4 v[8:11], v[12:13], off nt
    buffer_store_dwordx2 v[14:15], v16, s[4:7], 0 offen nt
    s_waitcnt vmcnt(2)
    s_barrier
    global_atomic_add v17, v18, s[8:9]
    s_endpgm
""")


def test_count_one_too_loose_fails():
    assert not _run("""
    buffer_store_dwordx4 v[0:3], v4, s[0:3], 0 offen
    global_load_dwordx4 v[8:11], v[12:13], off nt
    buffer_store_dwordx2 v[14:15], v16, s[4:7], 0 offen nt
    s_waitcnt vmcnt(3)
    global_atomic_add v17, v18, s[8:9]
    s_endpgm
""")


@pytest.mark.parametrize("marker", ["", "; %bb.1:\n"])
def test_branch_around_the_wait_fails(marker):
    # one path waits, the other jumps straight to the publish; LLVM marks the
    # fall-through block with a comment only, or with nothing
    assert not _run(f"""
    buffer_store_dwordx4 v[0:3], v4, s[0:3], 0 offen
    s_cbranch_scc1 .LBB0_2
{marker}    s_waitcnt vmcnt(0)
.LBB0_2:
    s_barrier
    global_atomic_add v17, v18, s[8:9]
    s_endpgm
""")


def test_wait_on_both_branches_passes():
    assert _run("""
    buffer_store_dwordx4 v[0:3], v4, s[0:3], 0 offen
    s_cbranch_scc1 .LBB0_2
; %bb.1:
    s_waitcnt vmcnt(0)
    s_branch .LBB0_3
.LBB0_2:
    global_load_dword v5, v[12:13], off nt
    s_waitcnt vmcnt(1)
.LBB0_3:
    s_barrier
    global_atomic_add v17, v18, s[8:9]
    s_endpgm
""")


def test_wait_after_the_barrier_fails():
    # wave 0's add publishes every wave's stores: a wait between the barrier and the add
    # covers the adding wave only
    assert not _run("""
    buffer_store_dwordx4 v[0:3], v4, s[0:3], 0 offen
    s_barrier
    s_waitcnt vmcnt(0)
    global_atomic_add v17, v18, s[8:9]
    s_endpgm
""")


def test_relaxed_far_branch_fails():
    # s_getpc/s_add/s_setpc (LLVM branch relaxation): an edge the CFG walk cannot see
    assert not _run("""
    buffer_store_dwordx4 v[0:3], v4, s[0:3], 0 offen
    s_waitcnt vmcnt(0)
    s_barrier
    s_getpc_b64 s[10:11]
    s_add_u32 s10, s10, 0x40
    s_addc_u32 s11, s11, 0
    s_setpc_b64 s[10:11]
    global_atomic_add v17, v18, s[8:9]
    s_endpgm
""")


@pytest.mark.parametrize("wait", [True, False])
def test_relaxed_far_branch_is_followed(wait):
    # LLVM's relaxed form of a far branch: its target edge is followed like an s_branch, so a
    # relaxed branch around the wait is caught and one through it passes
    w = "    s_waitcnt vmcnt(0)\n" if wait else ""
    assert _run(f"""
    buffer_store_dwordx4 v[0:3], v4, s[0:3], 0 offen
{w}    s_cbranch_scc0 .LBB0_12
; %bb.9:
    s_getpc_b64 s[98:99]
.Lpost_getpc0:
    s_add_u32 s98, s98, (.LBB0_20-.Lpost_getpc0)&4294967295
    s_addc_u32 s99, s99, (.LBB0_20-.Lpost_getpc0)>>32
    s_setpc_b64 s[98:99]
.LBB0_12:
    s_waitcnt vmcnt(0)
.LBB0_20:
    s_barrier
    global_atomic_add v17, v18, s[8:9]
    s_endpgm
""") == wait


def test_policy_stores_are_not_slot_stores():
    # RD rows are stored with a cache policy (nt / sc1): nothing to prove for them
    assert _run("""
    buffer_store_dwordx2 v[0:1], v4, s[0:3], 0 offen nt
    buffer_store_dwordx2 v[0:1], v4, s[0:3], 0 offen sc1
    global_atomic_add v17, v18, s[8:9]
    s_endpgm
""")


def test_built_kernel_passes():
    s = os.path.join(ROOT, "fmcw_radar_processing_amd", "csrc", "build", "kernels_xcd.s")
    if not os.path.exists(s):
        pytest.skip("libfmcw not built here (build() writes build/kernels_xcd.s)")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_vmcnt.py"), s],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "uncovered" not in r.stdout
