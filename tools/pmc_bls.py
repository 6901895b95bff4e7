"""BLS kernel rooflines from one rocprofv3 --pmc pass of tools/bls_prof.sh (SQ_WAVES,
SQ_INSTS_VALU, SQ_INSTS_VALU_INT64, SQ_WAVE_CYCLES, SQ_ACTIVE_INST_VALU, ...): for each bls_*
kernel, per dispatch, the executed v_mad_u64_u32-class instructions (SQ_INSTS_VALU_INT64, wave
level) x 64 lanes / kernel duration (the same dispatches' timestamps), against the MAD64 peak;
and the per-wave VALU issue rate (what bounds a latency-critical pairing check: a lone wave
per SIMD issues one instruction every few cycles).  Writes the JSON bench.py attaches to its
bls_config4 record (profiles/r02_pmc_bls.json).

usage: python tools/pmc_bls.py gpurun_out/blsprof/pmc1/run_counter_collection.csv > profiles/r02_pmc_bls.json
"""
import csv
import json
import sys
from collections import defaultdict

CLOCK_HZ = 2.4e9
SIMDS = 256 * 4
MAD64_PEAK = 256 * 4 * 16 * CLOCK_HZ  # lane-mads/s: v_mad_u64_u32 at half the INT32 rate (32 lanes/clk/SIMD)


def main():
    path = sys.argv[1]
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter sums
    span = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not name.startswith("bls_"):
            continue
        key = (name, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        span[key] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    kern = defaultdict(list)
    for (name, d), c in per.items():
        t0, t1 = span[(name, d)]
        kern[name].append((c, (t1 - t0) * 1e-9, int(d)))
    out = {"source": "rocprofv3 --pmc (one pass) over tools/bls_probe.py --reps 1, config #4 (n=1024, k=683)",
           "mad64_peak_lane_ops_per_s": MAD64_PEAK, "clock_hz": CLOCK_HZ, "kernels": {}}
    for name, rows in sorted(kern.items()):
        # the longest dispatch of each kernel is the config #4 call (parse-only and small calls are shorter)
        c, dt, d = max(rows, key=lambda x: x[1])
        waves = c.get("SQ_WAVES", 0.0)
        i64 = c.get("SQ_INSTS_VALU_INT64", 0.0)
        valu = c.get("SQ_INSTS_VALU", 0.0)
        cyc = c.get("SQ_WAVE_CYCLES", 0.0) * 4  # counter ticks every 4 cycles (gfx9)
        rec = {"dispatch": d, "duration_ms": dt * 1e3, "waves": waves,
               "int64_wave_insts": i64, "valu_wave_insts": valu,
               "mad_lane_ops_per_s": i64 * 64 / dt if dt > 0 else None}
        rec["mad_frac_of_peak"] = rec["mad_lane_ops_per_s"] / MAD64_PEAK if dt > 0 else None
        if waves:
            rec["valu_insts_per_wave"] = valu / waves
            rec["wave_cycles_per_valu"] = cyc / valu if valu else None
            rec["simd_occupancy"] = min(1.0, waves / SIMDS)
        out["kernels"][name] = rec
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
