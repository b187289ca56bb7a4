#!/usr/bin/env python3
"""Simulate rt_render_screen's chunk schedule (rt_screen.cpp) on the reference's own per-pixel sample counts
(from the oracle's rayTraceScreen): round trips on the critical path, rays traced, dropped continuations.
The actual stream position of a pixel is the prefix sum of the counts, so the schedule depends on nothing else.
usage: screen_sim.py [scene W H] [--win 56] [--next 1] [--conf 0]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counts_for(name, W, H):
    cache = f"/tmp/screen_counts_{name}_{W}x{H}.npy"
    if os.path.exists(cache):
        return np.load(cache)
    from oracle import pyoracle as po
    from ray_tracer_fragment_shader_amd import scenes
    sa = scenes.CONFIGS[name].scene().to_abi()
    _, ns, _ = po.render_screen(sa, W, H, 5, po.GLIBC, 1)
    ns = ns.reshape(-1).astype(np.int64)
    np.save(cache, ns)
    return ns


def simulate(cnt, W, win=28, next_mul=1, conf=0, max_pix=4096, max_rays=1 << 19):
    P = len(cnt)
    start = np.concatenate([[0], np.cumsum(cnt)])          # actual first sample of each pixel
    counts = np.zeros(P, np.int64)                           # resolved
    pcount = np.zeros(P, np.int64)
    st = {"trips": 0, "rays": 0, "chunks": 0, "dropped": 0}

    def predict(pix, p):
        below = pix - W
        if below >= 0:
            return counts[below] if below < p else pcount[below]
        return counts[p - 1] if p > 0 else 16

    def window(pix, p, pred, q):
        if not conf or q == 0:                              # a chunk's first pixel always resolves
            return win, win
        # confident: the three resolved pixels below agree (and the one left of them), narrow window
        below = pix - W
        if below - 1 >= 0 and below + 1 < p:
            b = counts[below - 1:below + 2]
            if b[0] == b[1] == b[2]:
                return conf, conf
        return win, win

    def queue(p0, pred_start, floor, want, p):
        S0 = max(floor, pred_start - win if pred_start > win else 0)
        m = min(want, P - p0)
        spred = pred_start - S0
        pix_w = []
        total = 0
        for q in range(m):
            pix = p0 + q
            pred = predict(pix, p)
            wl, wh = window(pix, p, pred, q)
            lo = max(0, spred - wl)
            hi = max(lo, spred + pred + wh)
            if total + hi - lo > max_rays or hi > max_pix * 16 + 2 * win + 16:
                m = q
                break
            pcount[pix] = pred
            pix_w.append((lo, hi))
            total += hi - lo
            spred += pred
        st["rays"] += total
        st["chunks"] += 1
        return {"p0": p0, "m": m, "S0": S0, "w": pix_w, "spred_end": spred}

    p, chunk = 0, 64
    cur = queue(0, 0, 0, chunk, 0)
    while p < P:
        nxt = None
        if next_mul > 0 and cur["p0"] + cur["m"] < P:
            nxt = queue(cur["p0"] + cur["m"], cur["S0"] + cur["spred_end"], start[p],
                        min(chunk * next_mul, max_pix), p)
        st["trips"] += 1
        q, broke = 0, False
        while q < cur["m"]:
            pix = cur["p0"] + q
            A = start[pix] - cur["S0"]                       # actual position, relative to the chunk
            lo, hi = cur["w"][q]
            if A < lo or A + cnt[pix] > hi:
                broke = True
                break
            counts[pix] = cnt[pix]
            q += 1
        p = cur["p0"] + q
        if not broke and q == cur["m"]:
            chunk = min(max_pix, chunk * 2)
            if nxt is not None:
                cur = nxt
            elif p < P:
                cur = queue(p, start[p], start[p], chunk, p)
            continue
        chunk = max(16, chunk // 2)
        if nxt is not None:
            st["dropped"] += 1
        if p < P:
            cur = queue(p, start[p], start[p], chunk, p)
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene", nargs="*", default=["demo", "500", "500"])
    ap.add_argument("--win", type=int, default=56)
    ap.add_argument("--next", type=int, default=1)
    ap.add_argument("--conf", type=int, default=0)
    a = ap.parse_args()
    name, W, H = a.scene[0], int(a.scene[1]), int(a.scene[2])
    cnt = counts_for(name, W, H)
    st = simulate(cnt, W, a.win, a.next, a.conf)
    st["samples"] = int(cnt.sum())
    print(st)


if __name__ == "__main__":
    main()
