"""Summarises the stall PMC passes of scripts/gpu_pmc_stall.sh (gpurun_out/pmc11, pmc12):
per-launch counter means of k_viterbi3 and k_data_fft and their fractions of wave cycles.
usage: python scripts/pmc_stall_summary.py OUT.json"""
import csv
import json
import sys
from collections import defaultdict

sys.path.insert(0, ".")
from ziria_amd.build import source_hash  # noqa: E402

KERNELS = {"k_viterbi3<0, false>": "k_viterbi3", "k_data_fft<false>": "k_data_fft", "k_descramble_crc": "k_descramble_crc",
           "k_signal_vit": "k_signal_vit", "k_signal_fft<false>": "k_signal_fft", "k_pkt_plan": "k_pkt_plan"}
vals = defaultdict(lambda: defaultdict(list))
for i in (11, 12):
    for r in csv.DictReader(open(f"gpurun_out/pmc{i}/pmc_counter_collection.csv")):
        for pat, name in KERNELS.items():
            if pat in r["Kernel_Name"]:
                vals[name][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
out = {"source": f"scripts/gpu_pmc_stall.sh (bench.py --steps 1 --warmup 1 --pipeline 1), sources {source_hash()[:8]}",
       "kernels": {}}
for name, d in vals.items():
    per = defaultdict(list)
    for (c, _), v in d.items():
        per[c].append(sum(v))                           # summed over the dispatch's XCC rows
    cnt = {c: round(sum(v) / len(v)) for c, v in per.items()}
    wc = cnt.get("SQ_WAVE_CYCLES", 0) or 1
    fr = {c: round(cnt[c] / wc, 3) for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                             "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS") if c in cnt}
    out["kernels"][name] = {"counters_per_launch": cnt, "fractions_of_wave_cycles": fr}
json.dump(out, open(sys.argv[1], "w"), indent=1)
print(json.dumps({k: v["fractions_of_wave_cycles"] for k, v in out["kernels"].items()}))
