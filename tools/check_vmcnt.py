"""Build-time proof of k_rdx's hand-off publish on the code the compiler emitted.

k_rdx (kernels_xcd.hip) publishes a frame's range-cube slot with one relaxed
agent-scope atomic add after every wave waited (``s_waitcnt vmcnt(N)``) for its
slot stores and a workgroup barrier.  N is counted by hand: the operations the
wave issued AFTER its slot stores (chirp loads, profile and RD stores) may stay
in flight.  ``s_waitcnt vmcnt(N)`` waits until at most the wave's N youngest
vector-memory operations are outstanding (they complete in issue order,
MI355X_MICROARCH.md), so a slot store is known complete at a wait exactly when
at least N vector-memory operations were issued after it and before the wait.

This script reads the gfx950 assembly of every k_rdx instantiation and checks,
on every control-flow path into every no-return ``global_atomic_add`` (the
publishes), that each slot store -- a ``buffer_store_*`` without a cache-policy
flag; k_rdx issues no other such stores -- is covered by some wait on the way: between the store and
that wait at least N vector-memory operations were issued.  A path with no
slot store (the first steps) is fine.  Wave 0's add publishes every wave's stores, so a wait
counts only when it comes BEFORE the last ``s_barrier`` ahead of the publish (every wave
runs the same code: its wait then precedes the barrier wave 0 crosses before adding); a
wait between that barrier and the add covers the adding wave alone.  Calls are treated
as issuing nothing and waiting for nothing (conservative), and an ``s_setpc_b64`` inside
a k_rdx body (branch relaxation of a far branch: a CFG edge this script cannot follow)
fails the check.  Exit status 1 on any uncovered path:
the Makefile then fails the build, so a compiler change that splits, merges or
reorders a store cannot silently publish a slot before its bytes are in L2.

  python tools/check_vmcnt.py kernels_xcd.s [--quiet]
"""
from __future__ import annotations

import re
import sys

INF = float("inf")
RE_LABEL = re.compile(r"^(\.LBB\d+_\d+|[A-Za-z_][\w.$]*):")
RE_VMCNT = re.compile(r"vmcnt\((\d+)\)")
RE_BB = re.compile(r"^;\s*(%bb\.\d+):")


def functions(text: str, pattern: str):
    """{name: [lines]} of the functions whose symbol matches pattern."""
    out, cur, name = {}, None, None
    for ln in text.splitlines():
        s = ln.strip()
        m = RE_LABEL.match(s)
        if m and not s.startswith(".L") and re.search(pattern, m.group(1)):
            name, cur = m.group(1), []
            out[name] = cur
            continue
        if cur is not None:
            if s.startswith(".Lfunc_end"):
                cur, name = None, None
                continue
            cur.append(s)
    return out


def blocks(lines):
    """[(label, [instr])] in layout order; instructions without comments/directives.

    A block starts at every ``.LBB`` label, at every fall-through block LLVM marks
    only with a ``; %bb.N:`` comment, and after every branch or end: a conditional
    branch is always the last instruction of its block, so cfg() sees both edges.
    """
    bl = [("entry", [])]
    for s in lines:
        m = RE_LABEL.match(s)
        if m and s.startswith(".LBB"):
            bl.append((m.group(1), []))
            continue
        m = RE_BB.match(s)
        if m:
            bl.append((m.group(1), []))
            continue
        s = s.split(";")[0].strip()
        if not s or s.startswith("."):
            continue
        bl[-1][1].append(s)
        op = s.split()[0]
        if op == "s_branch" or op.startswith("s_cbranch") or op in ("s_endpgm", "s_setpc_b64"):
            bl.append((f"{bl[-1][0]}+", []))
    return bl


def is_slot_store(ins: str) -> bool:
    if not ins.startswith("buffer_store"):
        return False
    flags = ins.split()[1:]
    return not any(f in ("sc0", "sc1", "nt", "glc", "slc") for f in flags)


def is_vmem(ins: str) -> bool:
    op = ins.split()[0]
    return op.startswith(("global_", "buffer_", "scratch_", "flat_")) and op not in ("buffer_inv",)


RE_RELAX = re.compile(r"^s_add_u32\s+(s\d+),\s*\1,\s*\((\.LBB\d+_\d+)-\.Lpost_getpc\d+\)")


def relaxed_target(ins):
    """Target label of LLVM's relaxed far branch (s_getpc_b64 s[a:b]; s_add_u32 sa, sa,
    (.LBBx_y-.Lpost_getpcN)&...; s_addc_u32; s_setpc_b64 s[a:b]) ending the block, else None."""
    if not ins or not ins[-1].startswith("s_setpc_b64"):
        return None
    reg = re.search(r"s\[(\d+):\d+\]", ins[-1])
    for s in reversed(ins[:-1]):
        m = RE_RELAX.match(s)
        if m and reg and m.group(1) == f"s{reg.group(1)}":
            return m.group(2)
    return None


def cfg(bl):
    idx = {lab: i for i, (lab, _) in enumerate(bl)}
    succ = []
    for i, (_, ins) in enumerate(bl):
        last = ins[-1].split() if ins else []
        op = last[0] if last else ""
        nxt = [i + 1] if i + 1 < len(bl) else []
        if op == "s_branch":
            succ.append([idx[last[1]]])
        elif op == "s_setpc_b64" and relaxed_target(ins) in idx:
            succ.append([idx[relaxed_target(ins)]])     # a relaxed far branch: s_branch in effect
        elif op.startswith("s_cbranch"):
            succ.append([idx[last[1]]] + nxt)
        elif op in ("s_endpgm", "s_setpc_b64"):
            succ.append([])
        else:
            succ.append(nxt)
    pred = [[] for _ in bl]
    for i, ss in enumerate(succ):
        for j in ss:
            pred[j].append(i)
    return pred


def check_function(name, lines, quiet=False):
    bl = blocks(lines)
    pred = cfg(bl)
    pubs = [(b, k) for b, (_, ins) in enumerate(bl) for k, s in enumerate(ins)
            if s.startswith("global_atomic_add") and " sc0" not in s and " glc" not in s]
    stores = sum(1 for _, ins in bl for s in ins if is_slot_store(s))
    unresolved = [lab for lab, ins in bl if ins and ins[-1].startswith("s_setpc_b64") and relaxed_target(ins) is None]
    if unresolved:
        if not quiet:
            print(f"{name}: s_setpc_b64 in block {unresolved[0]} with no s_getpc/s_add_u32 target: "
                  "the CFG is not followed, FAIL")
        return False
    bad = []
    worst = {}
    for b0, k0 in pubs:
        # backward search; state = the smallest "still needed" count over the waits passed
        # (larger = worse) and whether the walk has crossed an s_barrier yet (only waits behind
        # one count); a block is re-walked only with a worse state than before
        best = {}
        work = [(b0, k0, INF, False, ())]
        while work:
            b, k, rem, crossed, path = work.pop()
            ins = bl[b][1]
            hit = False
            for i in range(k - 1, -1, -1):
                s = ins[i]
                if s.startswith("s_barrier"):
                    crossed = True
                m = RE_VMCNT.search(s) if s.startswith("s_waitcnt") else None
                if m and crossed:
                    rem = min(rem, int(m.group(1)))
                if is_slot_store(s):
                    if rem > 0:
                        bad.append((bl[b0][0], bl[b][0], rem, path + (bl[b][0],)))
                    worst[(b0, k0)] = max(worst.get((b0, k0), -INF), rem)
                    hit = True
                    break
                if is_vmem(s) and rem != INF:
                    rem -= 1
            if hit:
                continue
            for p in pred[b]:
                if (p, crossed) in best and best[(p, crossed)] >= rem:
                    continue
                best[(p, crossed)] = rem
                work.append((p, len(bl[p][1]), rem, crossed, (path + (bl[b][0],))[-6:]))
    if not quiet:
        margins = ",".join("-" if (b, k) not in worst else
                           "none" if worst[(b, k)] == INF else str(int(-worst[(b, k)])) for b, k in pubs)
        print(f"{name}: {len(pubs)} publish atomics (margins {margins}), {stores} slot stores, "
              f"{'OK' if not bad else str(len(bad)) + ' uncovered path(s)'}")
    for pub, blk, rem, path in bad[:5]:
        print(f"  publish in {pub}: slot store in {blk} not covered (needs {rem} more ops); path ...{' <- '.join(path)}")
    return not bad and (stores == 0 or pubs)


def main(argv):
    quiet = "--quiet" in argv
    paths = [a for a in argv if not a.startswith("--")]
    ok = True
    n = 0
    for path in paths:
        fns = functions(open(path).read(), r"k_rdx")
        n += len(fns)
        for name, lines in fns.items():
            ok &= bool(check_function(name, lines, quiet))
    if n == 0:
        print("check_vmcnt: no k_rdx function found", file=sys.stderr)
        return 1
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
