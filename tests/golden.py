"""Helpers for the committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def frames(cfg_name):
    return dict(np.load(os.path.join(GOLDEN, f"frames_{cfg_name}.npz")))


def kat(scene_name):
    return dict(np.load(os.path.join(GOLDEN, f"kat_{scene_name}.npz")))


def tree(case_name):
    """Ray-tree fixtures (scenes.TREE_CASES, make_golden.py make_tree)."""
    return dict(np.load(os.path.join(GOLDEN, f"tree_{case_name[5:]}.npz")))


def canonical_nan(a):
    """NaNs replaced by the default quiet NaN (payloads are not part of the parity contract)."""
    a = np.array(a, np.float64, copy=True)
    a[np.isnan(a)] = np.nan
    return a


def screen():
    """Reference-faithful rayTraceScreen pins (tests/golden/make_golden_screen.py)."""
    with open(os.path.join(GOLDEN, "screen.json")) as f:
        return json.load(f)
