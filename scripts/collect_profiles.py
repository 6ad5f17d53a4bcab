"""Copy a gpu_round.sh run's evidence from gpurun_out/ into profiles/rNN/ (tag given) and refresh
profiles/traffic.json from the two PMC passes (FETCH_SIZE x2 on gfx950, WRITE_SIZE as is).
Usage: python scripts/collect_profiles.py r01 v9 "kernel description" """
import csv
import collections
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd, tag, desc = sys.argv[1], sys.argv[2], sys.argv[3]
src = os.path.join(REPO, "gpurun_out")
dst = os.path.join(REPO, "profiles", rnd)
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "prof", "kt_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench_full.json"))


def per_dispatch(name):
    d = collections.defaultdict(float)
    rows = []
    for r in csv.DictReader(open(os.path.join(src, "prof", f"{name}_counter_collection.csv"))):
        if "turbo_decode" in r["Kernel_Name"] or "demux" in r["Kernel_Name"]:
            rows.append(r)
        if "turbo_decode" in r["Kernel_Name"]:
            d[r["Dispatch_Id"]] += float(r["Counter_Value"])
    with open(os.path.join(dst, f"{tag}_pmc_{name}.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    return list(d.values())


f, w = per_dispatch("fetch"), per_dispatch("write")
fk, wk = sum(f) / len(f), sum(w) / len(w)
path = os.path.join(REPO, "profiles", "traffic.json")
rec = json.load(open(path))
r = rec["K6144_B4096_it8_f64_logmap"]
r.update(fetch_size_kib_raw=fk, write_size_kib_raw=wk, fetch_bytes=int(fk * 1024 * 2), write_bytes=int(wk * 1024),
         launches=len(f), kernel=f"{tag} ({desc})",
         source="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-trace of bench.py "
                f"--steps 8 --warmup 1; profiles/{rnd}/{tag}_pmc_*.csv")
r["bytes_per_launch"] = r["fetch_bytes"] + r["write_bytes"]
json.dump(rec, open(path, "w"), indent=1)
print(json.dumps(r, indent=1))
