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


def screen():
    """Reference-faithful rayTraceScreen pins (tests/golden/make_golden_screen.py)."""
    with open(os.path.join(GOLDEN, "screen.json")) as f:
        return json.load(f)
