"""Rounds per line of the small-batch line-cut search for candidate grid shapes, from the oracle's
per-line move strings (tools/cut_moves.py): a round walks from the centre while the position is
interior (all 8 neighbours on the grid).  profiles/r05_cutw/grid_shapes.txt is its output."""
import itertools
import sys
paths = [l.strip() for l in open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/gfplo_cut_paths.txt")]
MV = {str((s0 + 1) * 3 + (s1 + 1)): (s0, s1) for s0 in (-1, 0, 1) for s1 in (-1, 0, 1)}
def rounds(cells, maxsteps=99):
    cells = set(cells)
    dec = {p for p in cells if all((p[0] + a, p[1] + c) in cells for a in (-1, 0, 1) for c in (-1, 0, 1))}
    tot = 0
    for pth in paths:
        mv = [MV[ch] for ch in pth] + [None]   # None: the final decision (stay)
        i = 0
        while i < len(mv):
            tot += 1
            pos = (0, 0); n = 0
            while i < len(mv) and pos in dec and n < maxsteps:
                m = mv[i]; i += 1; n += 1
                if m is None: break
                pos = (pos[0] + m[0], pos[1] + m[1])
    return tot / len(paths)
sq = [(a, c) for a in range(-1, 7) for c in range(-1, 7)]
print("8x8 (-1..6), 5 steps", rounds(sq, 5), "unlimited", rounds(sq))
for w in range(2, 5):
    band = [(a, a + d) for a in range(-1, 20) for d in range(-w, w + 1)]
    band = sorted(band, key=lambda p: (p[0] + p[1], abs(p[0]-p[1])))
    print("band |d|<=", w, "cells 64:", rounds(band[:64]), "cells 128:", rounds(band[:128]))
# 128-cell squares / rectangles
for (A, Cc) in [(8, 16), (16, 8), (11, 11), (12, 10)]:
    r = [(a, c) for a in range(-1, A - 1) for c in range(-1, Cc - 1)]
    print(f"{A}x{Cc}", len(r), rounds(r))
# triangle-ish: cells with a, c >= -1 and a + c <= K
for K in range(8, 16):
    t = [(a, c) for a in range(-1, 20) for c in range(-1, 20) if a + c <= K]
    print("tri K", K, len(t), rounds(t))
print("---- 64-cell families, unlimited steps")
best = []
for A in range(5, 14):
    for Cc in range(5, 14):
        for K in range(6, 26):
            cells = [(a, c) for a in range(-1, A) for c in range(-1, Cc) if a + c <= K]
            if len(cells) > 64: continue
            best.append((rounds(cells), A, Cc, K, len(cells)))
best.sort(); print(best[:8])
