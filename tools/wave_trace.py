#!/usr/bin/env python3
"""Per-wave timeline of one rt_render_kernel launch (diagnostic; needs the RT_WAVE_TRACE=1 build (copied over lib/librt_amd.so) from
tools/variants.sh, e.g. `bash tools/variants.sh trace=-DRT_WAVE_TRACE=1`).
Reports wave durations, concurrent waves over time (per XCD and total) and the tail.
usage: wave_trace.py [config]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    cfg = scenes.CONFIGS[name]
    W, H = cfg.width, cfg.height
    t = Tracer(0)
    t.set_scene(cfg.scene())
    bufs = t.alloc(W, H, rgba32f=True, rgba8=True)
    nwg = ((W + 7) // 8) * ((H + 7) // 8)
    tr = torch.zeros(nwg * 7, dtype=torch.int64, device="cuda")   # RT_WAVE_TRACE=2: + {tile row, cone, trace} stamps
    lib = abi.lib()
    lib.rt_debug_wave_trace.argtypes = [ctypes.c_void_p]
    for _ in range(3):
        t.render_into(cfg.camera(), W, H, cfg.depth, bufs)
    torch.cuda.synchronize()
    assert lib.rt_debug_wave_trace(ctypes.c_void_p(tr.data_ptr())) == 0
    t.render_into(cfg.camera(), W, H, cfg.depth, bufs)
    torch.cuda.synchronize()
    ab = tr.cpu().numpy()
    a = ab[: nwg * 4].reshape(nwg, 4)
    b = ab[nwg * 4:].reshape(nwg, 3)
    st, en, hw, md = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
    t0 = st.min()
    st, en, md = ((x - t0) * 10.0 / 1000.0 for x in (st, en, md))      # 100 MHz ticks -> us
    t_ty, t_cone, t_tr = ((x - t0) * 10.0 / 1000.0 for x in (b[:, 0], b[:, 1], b[:, 2]))
    dur = en - st
    hwid = hw & 0xFFFFFFFF
    xcc = (hw >> 32) & 0xF
    cu = (hwid >> 8) & 0xF
    se = (hwid >> 13) & 0x7
    simd = (hwid >> 4) & 0x3
    grid = np.linspace(0, en.max(), 41)
    conc = [int(((st <= x) & (en > x)).sum()) for x in grid]
    out = {
        "config": name, "waves": int(nwg), "span_us": round(float(en.max()), 2),
        "dur_us": {q: round(float(np.percentile(dur, q)), 2) for q in (5, 25, 50, 75, 95, 99, 100)},
        "mean_dur_us": round(float(dur.mean()), 3),
        "prologue_us": {q: round(float(np.percentile(md - st, q)), 2) for q in (5, 50, 95)},
        "mean_prologue_us": round(float((md - st).mean()), 3),
        "mean_to_tile_row_us": round(float((t_ty - st).mean()), 3) if b[:, 0].any() else None,
        "mean_to_cone_us": round(float((t_cone - st).mean()), 3) if b[:, 0].any() else None,
        "sum_dur_us_per_slot": round(float(dur.sum()) / (256 * 4 * 5), 2),
        "last_start_us": round(float(st.max()), 2),
        "p99_end_us": round(float(np.percentile(en, 99)), 2),
        "concurrency_over_time": conc,
        "xcc_counts": np.bincount(xcc, minlength=8).tolist(),
        "xcc_last_end_us": [round(float(en[xcc == k].max()), 2) if (xcc == k).any() else None for k in range(8)],
        "distinct_cu": int(len(set(zip(xcc.tolist(), se.tolist(), cu.tolist())))),
        "simd_counts": np.bincount(simd, minlength=4).tolist(),
    }
    # Attribution of the launch (r05): every wave slot over the span is either inside a wave phase or idle
    # (ramp: before the resident count first reaches 95% of its maximum; drain: after it last falls below; gaps).
    if b[:, 2].any():
        span = float(en.max())
        dt = 0.02
        tg = np.arange(0.0, span + dt, dt)
        ev_t = np.concatenate([st, en])
        ev_d = np.concatenate([np.ones_like(st), -np.ones_like(en)])
        o = np.argsort(ev_t, kind="stable")
        cum = np.cumsum(ev_d[o])
        conc_f = cum[np.searchsorted(ev_t[o], tg, side="right") - 1].astype(float)
        conc_f[tg < ev_t[o][0]] = 0.0
        cap = float(conc_f.max())
        full = np.nonzero(conc_f >= 0.95 * cap)[0]
        t_full, t_drop = tg[full[0]], tg[full[-1]]
        idle = (cap - conc_f) * dt
        phases = {"to_tile_row": float((t_ty - st).sum()), "tile_row_to_cone": float((t_cone - t_ty).sum()),
                  "cone_to_ray": float((md - t_cone).sum()), "trace": float((t_tr - md).sum()),
                  "stores": float((en - t_tr).sum())}
        att = {k: round(v / cap, 3) for k, v in phases.items()}
        att["idle_ramp"] = round(float(idle[tg < t_full].sum()) / cap, 3)
        att["idle_mid"] = round(float(idle[(tg >= t_full) & (tg <= t_drop)].sum()) / cap, 3)
        att["idle_drain"] = round(float(idle[tg > t_drop].sum()) / cap, 3)
        out["attribution_us"] = att                    # sums to the span: slot-us of each phase / resident maximum
        out["resident_max"] = int(cap)
        out["t_full_us"], out["t_drop_us"] = round(float(t_full), 2), round(float(t_drop), 2)
        out["mean_phase_us"] = {k: round(v / nwg, 3) for k, v in phases.items()}
        sky = dur <= np.percentile(dur, 50)
        out["trace_us_short_half"] = round(float((t_tr - md)[sky].mean()), 3)
        out["trace_us_long_half"] = round(float((t_tr - md)[~sky].mean()), 3)
    # duration by image row band (bottom = board rows)
    rows = (H + 7) // 8
    d2 = dur.reshape(rows, (W + 7) // 8)
    out["dur_by_tile_row_us"] = [round(float(x), 2) for x in d2.mean(axis=1)[:: max(1, rows // 16)]]
    print(json.dumps(out))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"wave_trace_{name}.npz"), start_us=st, end_us=en, hw=hw, mid_us=md,
             ty_us=t_ty, cone_us=t_cone, trace_us=t_tr,
             tiles_x=(W + 7) // 8, tiles_y=(H + 7) // 8)


if __name__ == "__main__":
    main()
