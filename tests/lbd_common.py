"""Synthetic keylines for the LBD tests (gfpl.synth_keylines)."""
import gfpl


def synth_keylines(n, w, h, seed, min_len=2.0, max_len=200.0, border=False):
    return gfpl.synth_keylines(n, w, h, seed, min_len, max_len, border)
