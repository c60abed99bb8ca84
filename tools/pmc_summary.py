"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the bench's GEMM launches into
per-launch HBM bytes (gfx950 correction: FETCH_SIZE counts half the bytes of wide coalesced
reads, so it is doubled; MI355X_MICROARCH.md 'HBM'). Writes profiles-ready JSON to stdout."""
import csv
import glob
import json
import os
import sys


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = list(csv.DictReader(open(f[0])))
    return rows


def per_kernel(rows, counter):
    out = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        name = r.get("Kernel_Name", "?")
        v = float(r["Counter_Value"])
        d = out.setdefault(name, [0.0, 0])
        d[0] += v
        d[1] += 1
    return out


fetch = per_kernel(load(sys.argv[1]), "FETCH_SIZE")
write = per_kernel(load(sys.argv[2]), "WRITE_SIZE")
res = {"unit": "bytes per launch", "fetch_correction": 2.0, "kernels": {}}
tot_b, tot_n = 0.0, 0
for k in sorted(set(fetch) | set(write)):
    f, nf = fetch.get(k, [0.0, 0])
    w, nw = write.get(k, [0.0, 0])
    n = max(nf, nw, 1)
    # rocprofv3 derived FETCH_SIZE / WRITE_SIZE are in KiB
    b = (2.0 * f + w) * 1024.0 / n
    res["kernels"][k[:80]] = {"launches": n, "fetch_kib": f / max(nf, 1), "write_kib": w / max(nw, 1),
                              "hbm_bytes_per_launch": b}
    tot_b += (2.0 * f + w) * 1024.0
    tot_n += n
res["family_hbm_bytes_per_launch"] = tot_b / max(tot_n, 1)
res["family_launches"] = tot_n
print(json.dumps(res, indent=1))
