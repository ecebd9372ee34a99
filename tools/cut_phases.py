#!/usr/bin/env python3
"""k_cut_search phase split from a bench clock dump (bench.py --dump-records X.npy with a library
built by `tools/build_variant.sh DIR -DGFPL_CUT_PCLOCK`): per search wave, shader-clock cycles in
the step evaluation + decision, exact rounds, bookkeeping and line transitions (slots 0-3), the
transitions' phases (slots 4-6), and the loop iterations / transitions counted (slot 7: n_it << 32 |
n_tr; the 8 sequences of a wave carry the wave's).

usage: python3 tools/cut_phases.py X_clk.npy [group size, default 8]
"""
import sys

import numpy as np


def main():
    clk = np.load(sys.argv[1])
    g = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    w = clk[::g].astype(np.float64)
    it_tr = clk[::g, 7].astype(np.int64)
    w = w[it_tr > 0]
    n_it, n_tr = (it_tr[it_tr > 0] >> 32).astype(np.float64), (it_tr[it_tr > 0] & 0xFFFFFFFF).astype(np.float64)
    names = ["step", "exact", "bookkeeping", "transition"]
    tot = w[:, :4].sum(axis=1)
    print(f"waves {len(w)}; cycles per wave: mean {tot.mean():.0f}, max {tot.max():.0f}")
    for i, n in enumerate(names):
        print(f"  {n:12s} {w[:, i].mean():12.0f}  {100 * w[:, i].sum() / tot.sum():5.1f} %")
    it, tr = n_it.mean(), n_tr.mean()
    print(f"iterations {it:.0f} per wave, transitions {tr:.0f}")
    for i, n in enumerate(["  info + record + S", "  open_line + prefetch", "  progress exchange"]):
        print(f"{n:24s} {w[:, 4 + i].mean() / max(tr, 1):8.0f} cycles per transition")
    print(f"cycles per iteration (step + exact + bookkeeping) {(w[:, 0] + w[:, 1] + w[:, 2]).mean() / it:.0f}; "
          f"per transition {w[:, 3].mean() / max(tr, 1):.0f}")


if __name__ == "__main__":
    main()
