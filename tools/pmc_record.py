"""Per-kernel PMC record from separate rocprofv3 --pmc passes (tools/pmc_passes.sh).

usage: python tools/pmc_record.py <dir holding pass*/**/*counter_collection.csv> <label> [kernel-prefix ...]

For every kernel whose name starts with one of the prefixes (default: all): each counter summed
over its per-XCD/SE instances within a dispatch, then averaged over the dispatches of the pass
(passes are separate runs of the same command, so every pass sees the same dispatches), plus:
  duration_ms            mean dispatch time in the passes (profiled runs clock lower: DVFS;
                         bench.py quotes its own HIP-event time as the roofline's basis)
  valu_insts_per_wave    SQ_INSTS_VALU / SQ_WAVES
  valu_active_frac       SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (per-wave issue share)
  issue_stall_frac       SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES       (dependency / pipe stalls)
  waitcnt_frac           SQ_WAIT_ANY / SQ_WAVE_CYCLES            (parked on s_waitcnt / barrier)
  wave_cycles_per_valu   4 x SQ_WAVE_CYCLES / SQ_INSTS_VALU      (counter ticks every 4 cycles)
  waves_per_simd         SQ_WAVES / 1,024 SIMDs
  mad_lane_ops_per_s     SQ_INSTS_VALU_INT64 x 64 / duration, and its fraction of the MAD64 peak
  hbm_bytes              (FETCH_SIZE x 2 + WRITE_SIZE) x 1,024: the x2 is the gfx950 correction for
                         16-B-per-lane reads (MI355X_MICROARCH.md, HBM section)
The record is stamped with the csrc tree hash (tools/tree_hash.py) so bench.py can tell a stale
record from a current one.  JSON on stdout."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tree_hash import csrc_tree_hash  # noqa: E402

SIMDS = 256 * 4
MAD64_PEAK = 256 * 4 * 16 * 2.4e9  # lane-mads/s: v_mad_u64_u32 at half the INT32 rate


def derive(c: dict, dur: float) -> dict:
    rec = {"duration_ms": dur * 1e3}
    rec.update(c)
    waves, valu, cyc = c.get("SQ_WAVES"), c.get("SQ_INSTS_VALU"), c.get("SQ_WAVE_CYCLES")
    if waves and valu:
        rec["valu_insts_per_wave"] = valu / waves
        rec["waves_per_simd"] = waves / SIMDS
    if cyc:
        for key, ctr in (("valu_active_frac", "SQ_ACTIVE_INST_VALU"), ("issue_stall_frac", "SQ_WAIT_INST_ANY"),
                         ("waitcnt_frac", "SQ_WAIT_ANY")):
            if ctr in c:
                rec[key] = c[ctr] / cyc
        if valu:
            rec["wave_cycles_per_valu"] = 4 * cyc / valu
    if "SQ_INSTS_VALU_INT64" in c and dur > 0:
        rec["mad_lane_ops_per_s"] = c["SQ_INSTS_VALU_INT64"] * 64 / dur
        rec["mad_frac_of_peak"] = rec["mad_lane_ops_per_s"] / MAD64_PEAK
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rec["hbm_bytes"] = (c["FETCH_SIZE"] * 2 + c["WRITE_SIZE"]) * 1024
    return rec


def main():
    args = sys.argv[1:]
    longest = "--longest" in args
    args = [a for a in args if a != "--longest"]
    root, label = args[0], args[1]
    prefixes = tuple(args[2:]) or ("",)
    # kernel -> pass -> dispatch id -> {counter: sum over instances}, and each dispatch's span
    calls = defaultdict(lambda: defaultdict(lambda: defaultdict(lambda: defaultdict(float))))
    spans = defaultdict(lambda: defaultdict(dict))
    files = sorted(glob.glob(f"{root}/pass*/**/*counter_collection.csv", recursive=True))
    if not files:
        sys.exit(f"no counter_collection.csv under {root}/pass*")
    for f in files:
        pass_id = f.split("/pass")[1].split("/")[0]
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            if not name.startswith(prefixes):
                continue
            d = int(r["Dispatch_Id"])
            calls[name][pass_id][d][r["Counter_Name"]] += float(r["Counter_Value"])
            spans[name][pass_id][d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {"label": label, "csrc_tree": csrc_tree_hash(), "passes": len(files),
           "selection": "the longest call of each kernel" if longest else "mean over the kernel's calls",
           "kernels": {}}
    for name in sorted(calls):
        # the j-th dispatch of a kernel is the same call in every pass (the passes rerun one program)
        per_pass = {p: sorted(ds) for p, ds in calls[name].items()}
        ncalls = min(len(v) for v in per_pass.values())
        merged = []
        for j in range(ncalls):
            c, durs = {}, []
            for p, ds in per_pass.items():
                c.update(calls[name][p][ds[j]])
                durs.append(spans[name][p][ds[j]])
            merged.append(derive(c, sum(durs) / len(durs) * 1e-9))
        if longest:
            rec = max(merged, key=lambda r: r["duration_ms"])
        else:
            keys = set().union(*merged)
            rec = {k: sum(r[k] for r in merged if k in r) / sum(1 for r in merged if k in r) for k in keys}
        rec["calls_per_pass"] = ncalls
        out["kernels"][name] = dict(sorted(rec.items()))
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
