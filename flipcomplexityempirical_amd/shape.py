"""District-shape observables: the ring cut edges of boundary_slope and the driver's slope
and angle.

The reference's "slope" updater (grid_chain_sec11.py:55-78; Frankenstein_chain.py:57-80)
collects the cut edges on the outer ring of the grid, and its driver (:371-394) takes the
first two of them, temp[0] and temp[1], and records once per yield

    enda, endb = midpoints of temp[0], temp[1]
    slope = (endb[1]-enda[1]) / (endb[0]-enda[0])     (np.Inf when endb[0] == enda[0])
    angle = arccos(clip(dot(anga/|anga|, angb/|angb|), -1, 1)),  anga = enda - (20, 20)

On the GPU (``Chains.enable_ring``) every chain keeps the pair (i, j) of its first two cut
ring edges in ring order and the kernels count yields per pair (fw_chains_enable_ring,
include/flipwalk.h); this module builds the ring of a graph from the reference's
predicates and turns the pair histogram into slopes and angles with the reference's own
float expressions, so the values are those of the reference formula bit for bit.
"""
from __future__ import annotations

from typing import Callable, Hashable, Tuple

import numpy as np

from .graph import Graph

Key = Hashable


def sec11_on_ring(last: int = 39) -> Callable[[Key, Key], bool]:
    """boundary_slope of grid_chain_sec11.py:55-78: both endpoints in row 0, column 0, row
    ``last`` or column ``last``, or one of the four corner diagonals (either orientation)."""
    diag = {((0, 1), (1, 0)), ((0, last - 1), (1, last)), ((last - 1, 0), (last, 1)),
            ((last - 1, last), (last, last - 1))}
    diag |= {(b, a) for a, b in diag}

    def on_ring(x0, x1) -> bool:
        return ((x0[0] == 0 and x1[0] == 0) or (x0[1] == 0 and x1[1] == 0) or
                (x0[0] == last and x1[0] == last) or (x0[1] == last and x1[1] == last) or
                (x0, x1) in diag)
    return on_ring


def frank_on_ring(m: int = 50) -> Callable[[Key, Key], bool]:
    """boundary_slope of Frankenstein_chain.py:57-80 (m = 50): both endpoints with first
    coordinate 0 or m-1, or second coordinate -m+1 or m (the diagonals are commented out)."""
    def on_ring(x0, x1) -> bool:
        return ((x0[0] == 0 and x1[0] == 0) or (x0[1] == -m + 1 and x1[1] == -m + 1) or
                (x0[0] == m - 1 and x1[0] == m - 1) or (x0[1] == m and x1[1] == m))
    return on_ring


def grid_on_ring(h: int, w: int) -> Callable[[Key, Key], bool]:
    """The same ring for a plain h x w grid (node keys (i, j)), without diagonals."""
    def on_ring(x0, x1) -> bool:
        return ((x0[0] == 0 and x1[0] == 0) or (x0[1] == 0 and x1[1] == 0) or
                (x0[0] == h - 1 and x1[0] == h - 1) or (x0[1] == w - 1 and x1[1] == w - 1))
    return on_ring


def ring_edges(g: Graph, on_ring: Callable[[Key, Key], bool]) -> Tuple[np.ndarray, np.ndarray]:
    """(ring_u, ring_w): the graph's edges (u < w, canonical CSR order = the ring order)
    whose node keys satisfy ``on_ring``."""
    e = g.edges()
    keys = g.nodes
    sel = np.array([on_ring(keys[u], keys[w]) for u, w in e.tolist()], bool)
    return np.ascontiguousarray(e[sel, 0]), np.ascontiguousarray(e[sel, 1])


def slope_and_angle_of(g: Graph, ring_u, ring_w, i: int, j: int, centre=(20, 20)):
    """The driver's slope and angle (grid_chain_sec11.py:374-394) for temp = [ring edge i,
    ring edge j], with the reference's expressions on the node keys."""
    temp = [(g.nodes[int(ring_u[i])], g.nodes[int(ring_w[i])]),
            (g.nodes[int(ring_u[j])], g.nodes[int(ring_w[j])])]
    enda = ((temp[0][0][0] + temp[0][1][0]) / 2, (temp[0][0][1] + temp[0][1][1]) / 2)
    endb = ((temp[1][0][0] + temp[1][1][0]) / 2, (temp[1][0][1] + temp[1][1][1]) / 2)
    if endb[0] != enda[0]:
        slope = (endb[1] - enda[1]) / (endb[0] - enda[0])
    else:
        slope = np.inf
    anga = (enda[0] - centre[0], enda[1] - centre[1])
    angb = (endb[0] - centre[0], endb[1] - centre[1])
    angle = np.arccos(np.clip(np.dot(anga / np.linalg.norm(anga), angb / np.linalg.norm(angb)),
                              -1, 1))
    return slope, float(angle)


def shape_samples(hist_ring: np.ndarray, g: Graph, ring_u, ring_w, centre=(20, 20)):
    """Pair histogram (FW_READ_HIST_RING) -> (slope[], angle[], count[], n_short): one
    entry per observed pair, with the yield count; n_short = yields with fewer than two cut
    ring edges (the reference raises IndexError on such a state)."""
    R = len(ring_u)
    h = np.asarray(hist_ring, np.uint64)
    idx = np.flatnonzero(h[:R * R])
    slopes = np.empty(len(idx))
    angles = np.empty(len(idx))
    for t, p in enumerate(idx):
        slopes[t], angles[t] = slope_and_angle_of(g, ring_u, ring_w, int(p) // R, int(p) % R,
                                                  centre)
    return slopes, angles, h[idx].astype(np.int64), int(h[R * R])


def shape_histograms(hist_ring, g: Graph, ring_u, ring_w, angle_bins=64, slope_bins=None,
                     centre=(20, 20)):
    """Yield-weighted histograms of the angle over [0, pi] and of arctan(slope) over
    [-pi/2, pi/2] (np.inf -> pi/2): the distributions behind the reference's slope.png /
    angle.png traces, summed over every chain of the handle."""
    s, a, c, _ = shape_samples(hist_ring, g, ring_u, ring_w, centre)
    ha, ea = np.histogram(a, bins=angle_bins, range=(0.0, np.pi), weights=c)
    hs, es = np.histogram(np.arctan(s), bins=slope_bins or angle_bins,
                          range=(-np.pi / 2, np.pi / 2), weights=c)
    return (ha.astype(np.int64), ea), (hs.astype(np.int64), es)
