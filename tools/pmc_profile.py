#!/usr/bin/env python3
"""profiles/pmc_<cfg>.json from a tools/pmc.sh summary (gpurun_out/pmc_<cfg>/summary.json).

usage: pmc_profile.py <cfg> <summary.json> [note]

Records, per launch of the dominant rt_render_kernel instance:
  * HBM bytes: WRITE_SIZE + 2 x FETCH_SIZE (KiB; gfx950 FETCH_SIZE counts half of wide coalesced reads,
    MI355X_MICROARCH.md HBM section) -> "hbm_bytes_per_launch" (bench.py's roofline.traffic);
  * issued FP64 work: (ADD_F64 + MUL_F64 + TRANS_F64 + 2 FMA_F64) wave-instructions x 64 lanes
    -> "fp64_flops_issued_per_launch" (an upper bound: lanes masked off by divergence are counted),
    which bench.py divides by the measured kernel time for roofline_fp64;
  * the instruction / wait mix when those counters were collected."""
import json
import sys

ALG_BYTES = {"c1": 160 * 120 * 20, "c2": 1920 * 1080 * 20, "c3": 3840 * 2160 * 20, "c5": 7680 * 4320 * 20}


def main():
    cfg, path = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    d = json.load(open(path))
    ks = [k for k in d if "rt_render_kernel" in k]
    k = max(ks, key=lambda x: d[x].get("_dispatches", 0))
    c = d[k]
    out = {"config": cfg, "kernel": k,
           "source": "rocprofv3 --pmc, one counter group per run (tools/pmc.sh), mean per dispatch",
           "correction": "gfx950 FETCH_SIZE counts half of wide coalesced reads (MI355X_MICROARCH.md HBM): read "
                         "bytes = 2 x FETCH_SIZE; WRITE_SIZE exact for 16-B/lane stores",
           "algorithmic_bytes_per_launch": ALG_BYTES.get(cfg)}
    if "WRITE_SIZE" in c and "FETCH_SIZE" in c:
        out["write_size_kib"] = c["WRITE_SIZE"]
        out["fetch_size_kib"] = c["FETCH_SIZE"]
        out["hbm_bytes_per_launch"] = c["WRITE_SIZE"] * 1024 + 2 * c["FETCH_SIZE"] * 1024
        if ALG_BYTES.get(cfg):
            out["hbm_ratio"] = round(out["hbm_bytes_per_launch"] / ALG_BYTES[cfg], 4)
    f64 = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"]
    if all(x in c for x in f64):
        wi = c[f64[0]] + c[f64[1]] + 2 * c[f64[2]] + c[f64[3]]
        out["fp64_wave_instructions"] = {x.replace("SQ_INSTS_VALU_", ""): c[x] for x in f64}
        out["fp64_flops_issued_per_launch"] = wi * 64
        if c.get("SQ_INSTS_VALU"):
            # FP64 share of the issued VALU wave-instructions (each FP64 instruction counted once)
            n64 = c[f64[0]] + c[f64[1]] + c[f64[2]] + c[f64[3]]
            out["fp64_share_of_valu"] = round(n64 / c["SQ_INSTS_VALU"], 4)
            out["valu_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1) if c.get("SQ_WAVES") else None
            out["fp64_per_wave"] = round(n64 / c["SQ_WAVES"], 1) if c.get("SQ_WAVES") else None
    for x in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
              "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "VALUBusy", "VALUUtilization", "GRBM_GUI_ACTIVE"):
        if x in c:
            out.setdefault("mix", {})[x] = c[x]
    if note:
        out["note"] = note
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
