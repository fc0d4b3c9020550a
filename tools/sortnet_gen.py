#!/usr/bin/env python3
"""Generator of the common-mode kernel's three-input sorting / selection networks.

Writes ``csrc/sortnet_gen.h`` (``python tools/sortnet_gen.py``; ``--check`` only verifies and prints
the op counts).  Every network is a list of ops on register indices:

  comparator  (2, a, b)     a <- min(a, b), b <- max(a, b)                      2 VALU (1 if one output is dead)
  3-sorter    (3, a, b, c)  a <- min3, b <- med3, c <- max3 of (a, b, c)        3 VALU (one per live output)

gfx950 has ``v_minimum3_f32`` / ``v_maximum3_f32`` / ``v_med3_f32``: a 3-sorter is three instructions
where three comparators are six, so networks are built from them where they pay:

* sorts: a merge tree whose leaves are 3-sorters and pairs, each internal node the cheaper of
  Batcher's odd-even merge and a mixed-radix bitonic merge (below), split points chosen by dynamic
  programming over the op count (44 values: 509 VALU instead of 694 for the odd-even merge sort);
* selections (the row medians): the backward cone of the sort of the two median ranks only
  (48 values, ranks 23 / 24: 434 VALU instead of the odd-even cone's 580);
* V-merges (the column phase's merge-split level): a V-shaped sequence (non-increasing, then
  non-decreasing) is sorted by cleaner levels of radix 2 or 3: at radix 3, position i, i + m,
  i + 2m of each block of 3m are 3-sorted, which leaves three V-shaped thirds in order (checked
  below for every 0-1 V-shaped input, hence for every input by the 0-1 principle).  44 values:
  165 VALU (radix 3 at every level over 81 virtual positions) instead of 224 for the radix-2 network.

Virtual +inf padding (positions past the real values) is tracked symbolically: an op against a pad
is a no-op or a relabelling, never an instruction.

Checks (every run): every merge node of every sort tree EXHAUSTIVELY on 0-1 inputs (a merge of
sorted runs of lengths a and b needs only the (a + 1)(b + 1) pairs of sorted 0-1 runs; with 3-sorter
and pair leaves this proves each whole sort by induction and the 0-1 principle, and a selection is
a backward cone of such a sort); sorts and selections also against ``sorted`` on random
permutations, inputs with duplicates and random 0-1 vectors; V-merges exhaustively on 0-1 V-shaped
inputs.  ``--check --diff`` also fails when the committed header differs from what this generator
writes (tests/test_sortnet_gen.py).
"""
from __future__ import annotations

import argparse
import functools
import itertools
import random
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
OUT = REPO / "csrc" / "sortnet_gen.h"
INF = None   # virtual +inf pad


def np2(n: int) -> int:
    p = 1
    while p < n:
        p <<= 1
    return p


def cost(ops) -> int:
    return sum(2 if o[0] == 2 else 3 for o in ops)


# ---- merges of two sorted label lists ---------------------------------------------------------
def oem_merge(a, b):
    """Batcher's odd-even merge of ascending label lists a, b (each padded with +inf to a power of 2)."""
    m = np2(max(len(a), len(b)))
    seq = list(a) + [INF] * (m - len(a)) + list(b) + [INF] * (m - len(b))
    ops = []

    def cmp(i, j):
        x, y = seq[i], seq[j]
        if y is INF:
            return
        if x is INF:   # +inf at the lower position: the comparator just swaps the labels
            seq[i], seq[j] = y, x
            return
        ops.append((2, x, y))

    def merge(lo, n, r):
        step = 2 * r
        if step < n:
            merge(lo, n, step)
            merge(lo + r, n, step)
            for i in range(lo + r, lo + n - r, step):
                cmp(i, i + r)
        else:
            cmp(lo, lo + r)

    merge(0, 2 * m, 1)
    return ops, [s for s in seq if s is not INF]


def cleaner_net(seq, radices):
    """Mixed-radix bitonic cleaner levels over a V-shaped / bitonic label sequence (INF = +inf pad)."""
    seq = list(seq)
    ops = []

    def group(pos):
        real = [seq[p] for p in pos if seq[p] is not INF]
        if len(real) == 2:
            ops.append((2, real[0], real[1]))
        elif len(real) == 3:
            ops.append((3, real[0], real[1], real[2]))
        for p, v in zip(pos, real + [INF] * (len(pos) - len(real))):
            seq[p] = v

    def rec(lo, n, lev):
        if n <= 1:
            return
        r = radices[lev]
        m = n // r
        for i in range(m):
            group([lo + i + k * m for k in range(r)])
        for k in range(r):
            rec(lo + k * m, m, lev + 1)

    rec(0, len(seq), 0)
    return ops, [s for s in seq if s is not INF]


def radix_plans(n: int):
    """(length, radices) of every 2^a 3^b >= n up to 2 np2(n), every order of the radices."""
    out = []
    for a in range(9):
        for b in range(6):
            L = 2 ** a * 3 ** b
            if n <= L <= 2 * np2(n):
                for perm in set(itertools.permutations([2] * a + [3] * b)):
                    out.append((L, list(perm)))
    return out


def best_cleaner(seq_real, layout):
    """Cheapest cleaner network for n real labels; layout(L) -> the padded sequence."""
    best = None
    for L, pl in radix_plans(len(seq_real)):
        ops, order = cleaner_net(layout(L), pl)
        if best is None or cost(ops) < cost(best[0]):
            best = (ops, order, (L, pl))
    return best


def b3_merge(a, b):
    """Merge of ascending a, b as the bitonic sequence a ++ (+inf pads) ++ reversed(b)."""
    n = len(a) + len(b)
    ops, order, _ = best_cleaner(list(a) + list(b), lambda L: list(a) + [INF] * (L - n) + list(reversed(b)))
    return ops, order


@functools.lru_cache(None)
def merge_cost(na: int, nb: int):
    a, b = list(range(na)), list(range(na, na + nb))
    c1 = cost(oem_merge(a, b)[0])
    c2 = cost(b3_merge(a, b)[0])
    return (c1, "oem") if c1 <= c2 else (c2, "b3")


@functools.lru_cache(None)
def sort_plan(n: int):
    """(op count, split, merge kind) of the cheapest merge tree with 3-sorter / pair leaves."""
    if n <= 1:
        return 0, None, None
    if n == 2:
        return 2, None, None
    if n == 3:
        return 3, None, None
    best = None
    for h in range(1, n // 2 + 1):
        mc, kind = merge_cost(h, n - h)
        c = sort_plan(h)[0] + sort_plan(n - h)[0] + mc
        if best is None or c < best[0]:
            best = (c, h, kind)
    return best


def tree_sort(idx):
    n = len(idx)
    if n == 1:
        return [], list(idx)
    if n == 2:
        return [(2, idx[0], idx[1])], list(idx)
    if n == 3:
        return [(3, idx[0], idx[1], idx[2])], list(idx)
    _, h, kind = sort_plan(n)
    o1, a = tree_sort(idx[:h])
    o2, b = tree_sort(idx[h:])
    om, order = oem_merge(a, b) if kind == "oem" else b3_merge(a, b)
    return o1 + o2 + om, order


def cone(ops, need):
    """Backward cone of the wires in `need`: ops with a live-output mask (dead ops dropped)."""
    need = set(need)
    out = []
    for op in reversed(ops):
        wires = op[1:]
        live = [w in need for w in wires]
        if not any(live):
            continue
        mask = sum(1 << i for i, l in enumerate(live) if l)
        out.append(op + (mask,))
        need.update(wires)
    return list(reversed(out))


def full_mask(ops):
    return [op + ((1 << (len(op) - 1)) - 1,) for op in ops]


def masked_cost(mops) -> int:
    return sum(bin(o[-1]).count("1") for o in mops)


# ---- evaluation / checks ----------------------------------------------------------------------
def run(mops, x):
    x = list(x)
    for o in mops:
        w, m = o[1:-1], o[-1]
        v = sorted(x[i] for i in w)
        for k, i in enumerate(w):
            if (m >> k) & 1:
                x[i] = v[k]
    return x


def check_sort(n, mops, order, trials=400):
    rng = random.Random(n)
    for t in range(trials):
        if t % 3 == 0:
            x = [rng.random() for _ in range(n)]
        elif t % 3 == 1:
            x = [rng.randint(0, 5) for _ in range(n)]
        else:
            x = [rng.randint(0, 1) for _ in range(n)]
        y = run(mops, x)
        if [y[i] for i in order] != sorted(x):
            return False
    return True


def check_select(n, mops, order, ranks, trials=2000):
    rng = random.Random(n + 1)
    for t in range(trials):
        x = [rng.random() for _ in range(n)] if t % 2 else [rng.randint(0, 3) for _ in range(n)]
        y = run(mops, x)
        s = sorted(x)
        if any(y[order[r]] != s[r] for r in ranks):
            return False
    return True


def merge_nodes(n):
    """(na, nb, kind) of every internal merge of tree_sort(n)'s tree."""
    if n <= 3:
        return []
    _, h, kind = sort_plan(n)
    return merge_nodes(h) + merge_nodes(n - h) + [(h, n - h, kind)]


def check_merge_exhaustive(na, nb, kind):
    """The merge network of sorted runs of lengths na, nb on every pair of sorted 0-1 runs."""
    a, b = list(range(na)), list(range(na, na + nb))
    ops, order = oem_merge(a, b) if kind == "oem" else b3_merge(a, b)
    mops = full_mask(ops)
    for i in range(na + 1):
        for j in range(nb + 1):
            v = [0] * i + [1] * (na - i) + [0] * j + [1] * (nb - j)
            y = run(mops, v)
            if [y[k] for k in order] != sorted(v):
                return False
    return True


def check_vmerge(n, mops, order):
    # every 0-1 V-shaped input 1^a 0^b 1^c: by the 0-1 principle the network sorts every V-shaped input
    for a in range(n + 1):
        for b in range(n + 1 - a):
            v = [1] * a + [0] * b + [1] * (n - a - b)
            y = run(mops, v)
            if [y[i] for i in order] != sorted(v):
                return False
    return True


# ---- the kernel's instances -------------------------------------------------------------------
SORTS = (4, 44, 64)          # column phase: per-lane sorts (M)
SELECTS = (8, 48, 64)        # row phase: median cones (L), ranks L/2 - 1, L/2 (toggle padding)
VMERGES = (4, 44, 64)        # column phase: V-shaped merge-split halves (M)


def sort_net(n):
    ops, order = tree_sort(list(range(n)))
    mops = full_mask(ops)
    for na, nb, kind in merge_nodes(n):
        assert check_merge_exhaustive(na, nb, kind), f"sort {n}: merge {na}+{nb} ({kind})"
    assert check_sort(n, mops, order), f"sort {n}"
    return mops, order


def select_net(n):
    ops, order = tree_sort(list(range(n)))
    for na, nb, kind in merge_nodes(n):
        assert check_merge_exhaustive(na, nb, kind), f"select {n}: merge {na}+{nb} ({kind})"
    pa, pb = (n - 1) // 2 if n & 1 else n // 2 - 1, ((n - 1) // 2 if n & 1 else n // 2 - 1) + 1
    mops = cone(ops, {order[pa], order[pb]})
    assert check_select(n, mops, order, (pa, pb)), f"select {n}"
    return mops, order, (pa, pb)


def vmerge_net(n):
    ops, order, plan = best_cleaner(list(range(n)), lambda L: list(range(n)) + [INF] * (L - n))
    mops = full_mask(ops)
    assert check_vmerge(n, mops, order), f"vmerge {n}"
    return mops, order, plan


def oem_sort_cost(n):
    ops = []
    P = np2(n)
    p = 1
    while p < P:
        k = p
        while k >= 1:
            j = k % p
            while j <= P - 1 - k:
                for i in range(0, min(k - 1, P - j - k - 1) + 1):
                    if (i + j) // (p * 2) == (i + j + k) // (p * 2) and i + j + k < n:
                        ops.append((2, i + j, i + j + k))
                j += 2 * k
            k //= 2
        p *= 2
    return ops


def emit(name, n, mops, order, note):
    lines = [f"// {note}", f"struct {name} {{", f"  static constexpr int kN = {n};",
             f"  static constexpr int kOps = {len(mops)};",
             f"  static constexpr int kValu = {masked_cost(mops)};",
             "  // output rank r of the sorted sequence sits in register kOut[r]",
             "  static constexpr short kOut[" + str(n) + "] = {" + ", ".join(str(v) for v in order) + "};",
             "  static constexpr NetOp kOp[" + str(len(mops)) + "] = {"]
    row = []
    for o in mops:
        w = list(o[1:-1]) + [0] * (3 - len(o[1:-1]))
        row.append(f"{{{len(o) - 2}, {w[0]}, {w[1]}, {w[2]}, {o[-1]}}}")
        if len(row) == 6:
            lines.append("      " + ", ".join(row) + ",")
            row = []
    if row:
        lines.append("      " + ", ".join(row) + ",")
    lines += ["  };", "};", ""]
    return lines


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true", help="verify and print op counts, write nothing")
    ap.add_argument("--diff", action="store_true", help="with --check: fail if csrc/sortnet_gen.h is stale")
    args = ap.parse_args()
    out = ["// GENERATED by tools/sortnet_gen.py -- do not edit.  Three-input sorting / selection networks",
           "// of the common-mode kernel (see the generator's docstring for the constructions and checks).",
           "#pragma once", "", "namespace pr {", "",
           "// kind 2: comparator (a, b); kind 3: 3-sorter (a, b, c); mask bit k: output k is live",
           "struct NetOp {", "  short kind, a, b, c, mask;", "};", "",
           "template <int N>", "struct GenSort {", "  static constexpr bool kHave = false;", "};",
           "template <int N>", "struct GenSelect {", "  static constexpr bool kHave = false;", "};",
           "template <int N>", "struct GenVMerge {", "  static constexpr bool kHave = false;", "};", ""]
    for n in SORTS:
        mops, order = sort_net(n)
        print(f"sort {n}: {masked_cost(mops)} VALU (odd-even merge sort {2 * len(oem_sort_cost(n))})")
        out += emit(f"GenSortNet{n}", n, mops, order, f"ascending sort of {n} registers")
        out += ["template <>", f"struct GenSort<{n}> : GenSortNet{n} {{", "  static constexpr bool kHave = true;",
                "};", ""]
    for n in SELECTS:
        mops, order, (pa, pb) = select_net(n)
        print(f"select {n} ranks {pa},{pb}: {masked_cost(mops)} VALU")
        out += emit(f"GenSelectNet{n}", n, mops, order,
                    f"registers kOut[{pa}], kOut[{pb}] <- the elements of rank {pa}, {pb} of {n} (other registers garbage)")
        out += ["template <>", f"struct GenSelect<{n}> : GenSelectNet{n} {{", "  static constexpr bool kHave = true;",
                f"  static constexpr int kRankA = {pa}, kRankB = {pb};", "};", ""]
    for n in VMERGES:
        mops, order, plan = vmerge_net(n)
        print(f"vmerge {n}: {masked_cost(mops)} VALU, {plan[0]} virtual positions, radices {plan[1]}")
        out += emit(f"GenVMergeNet{n}", n, mops, order,
                    f"ascending sort of a V-shaped sequence of {n} registers (radices {plan[1]} over {plan[0]})")
        out += ["template <>", f"struct GenVMerge<{n}> : GenVMergeNet{n} {{", "  static constexpr bool kHave = true;",
                "};", ""]
    out += ["}  // namespace pr", ""]
    text = "\n".join(out)
    if not args.check:
        OUT.write_text(text)
        print(f"wrote {OUT}")
    elif args.diff:
        if OUT.read_text() != text:
            raise SystemExit(f"{OUT} differs from the generator's output: regenerate it")
        print(f"{OUT} matches the generator")


if __name__ == "__main__":
    main()
