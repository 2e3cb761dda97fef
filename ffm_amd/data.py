"""Synthetic rooms and static floor fields.

Restates the recipe of the reference's ``create_12x12_map_and_sff.py:15-50``
(SoraKurihara/FFM) for any size: a one-cell wall border (value 2), one exit
(value 3) at ``(0, W // 2)``, free cells 0, and an L1 distance-to-exit static
floor field stored as float32 with ``inf`` on every non-passable cell.
``tests/test_data.py`` checks the 12x12 case against the files the reference's
own script writes (committed under ``tests/golden/``).
"""
from __future__ import annotations

import numpy as np

FREE, AGENT, WALL, EXIT = 0, 1, 2, 3


def make_room(H: int = 12, W: int = 12, exit_pos: tuple[int, int] | None = None) -> np.ndarray:
    """Map per ``create_12x12_map_and_sff.py:15-25`` scaled to H x W (uint8)."""
    if H < 3 or W < 3:
        raise ValueError("room needs at least 3x3 cells")
    m = np.zeros((H, W), dtype=np.uint8)
    m[0, :] = WALL
    m[-1, :] = WALL
    m[:, 0] = WALL
    m[:, -1] = WALL
    ex, ey = exit_pos if exit_pos is not None else (0, W // 2)
    m[ex, ey] = EXIT
    return m


def l1_sff(map_array: np.ndarray, dtype=np.float32) -> np.ndarray:
    """L1 distance to the nearest exit per ``create_12x12_map_and_sff.py:36-50``."""
    m = np.asarray(map_array)
    exits = np.argwhere(m == EXIT)
    H, W = m.shape
    xs, ys = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    d = np.full((H, W), np.inf, dtype=np.float64)
    for ex, ey in exits:
        d = np.minimum(d, np.abs(xs - ex) + np.abs(ys - ey))
    passable = (m == FREE) | (m == EXIT)
    out = np.where(passable, d, np.inf).astype(dtype)
    return out


def free_cells(map_array: np.ndarray) -> np.ndarray:
    """Row-major free-cell list, the order of ``np.argwhere(map == 0)``."""
    return np.flatnonzero(np.asarray(map_array).reshape(-1) == FREE)
