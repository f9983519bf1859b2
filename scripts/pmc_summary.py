"""Summarises rocprofv3 --pmc passes (scripts/gpu_pmc.sh) into per-kernel, per-launch
numbers for bench.py's roofline.traffic and the VALU evidence of DESIGN.md.

usage: python scripts/pmc_summary.py <dir with pmc1/ pmc2/ pmc3/ prof/> > pmc_summary.json

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): rocprofv3's FETCH_SIZE
and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16 B/lane
stores.  GRBM_GUI_ACTIVE is summed over the 8 XCDs.  SQ_INSTS_VALU counts wave64 VALU
instructions: x64 = lane operations, compared with the SIMD-32 peak of
256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T lane-ops/s over the kernel's traced time.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict

VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9


def short(name):
    """Kernel key: the function name, plus "_fix" for the seam-pass instantiation of
    k_viterbi3 (template <0, true>), whose launches are not the decode's."""
    m = re.search(r"zrx::(?:v\d::)?(\w+)(<[^>]*>)?", name)
    if not m:
        return name.split("(")[0][:60]
    k = m.group(1)
    if k == "k_viterbi3" and m.group(2) and "true" in m.group(2):
        k += "_fix"
    return k


def read_pmc(d):
    per = defaultdict(lambda: defaultdict(float))          # (kernel, dispatch) -> counter -> value
    durs = {}                                              # (kernel, dispatch) -> ns
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            key = (k, r.get("Dispatch_Id", "0"))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                durs[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = defaultdict(lambda: defaultdict(list))
    clk = defaultdict(list)                                # the shader clock of each dispatch, from its own
    for key, cs in per.items():                            # GRBM_GUI_ACTIVE and duration (8 XCDs)
        for c, v in cs.items():
            out[key[0]][c].append(v)
        if "GRBM_GUI_ACTIVE" in cs and durs.get(key):
            clk[key[0]].append(cs["GRBM_GUI_ACTIVE"] / 8 / durs[key])
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}, \
           {k: max(len(v) for v in cs.values()) for k, cs in out.items()}, clk


def read_trace(d):
    t = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            t[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return t


def main(root):
    counters, n, clocks = {}, {}, defaultdict(list)
    for p in sorted(glob.glob(os.path.join(root, "pmc*"))):
        if os.path.isdir(p):
            c, nn, ck = read_pmc(p)
            for k, v in c.items():
                counters.setdefault(k, {}).update(v)
                n[k] = max(n.get(k, 0), nn[k])
            for k, v in ck.items():
                clocks[k] += v
    trace = read_trace(os.path.join(root, "prof"))
    # The shader clock climbs from ~2.2 to 2.4 GHz over the first ~10 ms of load after an idle
    # GPU (profiles/r05/clock_probe.txt), so the trace's first launches run slower: the rates
    # below use the median launch (the steady clock the bench's timed steps run at); the mean
    # over every launch is kept beside it.
    dur = {k: statistics.median(v) for k, v in trace.items()}
    npkts = None
    for lg in glob.glob(os.path.join(root, "pmc*.log")):
        for line in open(lg):
            if line.startswith("{"):
                npkts = json.loads(line)["config"]["packets_per_gpu"]
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from ziria_amd.build import source_hash
    import subprocess
    try:
        rev = subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], text=True,
                                      stderr=subprocess.DEVNULL).strip()
    except (OSError, subprocess.CalledProcessError):
        rev = None
    res = {"npkts": npkts, "csrc_sha256": source_hash(), "git_head": rev,
           "source": "rocprofv3 --pmc, one timed step + one warmup of bench.py; durations from the "
                     "kernel-trace run of the default bench (rates use the median launch)",
           "kernels": {}}
    for k, cs in counters.items():
        if not k.startswith("k_"):
            continue
        e = {"dispatches": n[k], "counters": {c: round(v, 1) for c, v in cs.items()}}
        fetch = cs.get("FETCH_SIZE")
        write = cs.get("WRITE_SIZE")
        if fetch is not None and write is not None:
            e["fetch_bytes_corrected"] = fetch * 1024 * 2
            e["write_bytes"] = write * 1024
            e["hbm_bytes_per_launch"] = int(e["fetch_bytes_corrected"] + e["write_bytes"])
        if k in dur:
            e["avg_duration_ns"] = round(sum(trace[k]) / len(trace[k]), 1)
            e["median_duration_ns"] = round(dur[k], 1)
            e["trace_launches"] = len(trace[k])
            if "SQ_INSTS_VALU" in cs:
                lane_ops = cs["SQ_INSTS_VALU"] * 64
                e["valu_lane_ops_per_s"] = lane_ops / (dur[k] * 1e-9)
                e["valu_issue_frac_of_peak"] = round(e["valu_lane_ops_per_s"] / VALU_PEAK_LANE_OPS, 4)
            if "GRBM_GUI_ACTIVE" in cs:
                if clocks.get(k):                      # per dispatch of the PMC pass (its own durations)
                    e["effective_clock_ghz"] = round(statistics.mean(clocks[k]), 3)
                    e["effective_clock_ghz_range"] = [round(min(clocks[k]), 3), round(max(clocks[k]), 3)]
                if "SQ_ACTIVE_INST_VALU" in cs:
                    # gfx94x VALUBusy: SQ_ACTIVE_INST_VALU (quad-cycles) x 4 / SIMDs / GUI cycles
                    e["valu_busy"] = round(cs["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (cs["GRBM_GUI_ACTIVE"] / 8), 4)
        res["kernels"][k] = e
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
