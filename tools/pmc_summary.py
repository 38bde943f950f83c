"""Per-kernel HBM traffic from rocprofv3 PMC passes (one counter per pass: FETCH_SIZE, WRITE_SIZE).

  python tools/pmc_summary.py FETCH_CSV WRITE_CSV [--match k_pway] [--out profiles/traffic.json --tag-map JSON]

Groups dispatches by (kernel name, grid size), takes the median counter value per group and applies
the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE x 2 for 16-B-per-lane streaming reads
(the counter reports half the bytes of such a kernel), WRITE_SIZE as reported; both in KB (1024 B).
Prints one JSON line per group. With --out and --tag-map ({"tag": ["kernel substring", grid_size,
algorithmic_bytes]}), merges the matching groups into profiles/traffic.json under those tags.
"""
import argparse
import csv
import json
import statistics
import sys


def load(path, match):
    groups = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if match and match not in name:
                continue
            key = (name, int(row["Grid_Size"]))
            groups.setdefault(key, []).append(float(row["Counter_Value"]))
    return {k: statistics.median(v) for k, v in groups.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--match", default="k_")
    ap.add_argument("--out")
    ap.add_argument("--tag-map")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    fe, wr = load(a.fetch, a.match), load(a.write, a.match)
    rows = []
    for key in sorted(set(fe) & set(wr), key=lambda k: (k[0], k[1])):
        name, grid = key
        hbm = fe[key] * 2 * 1024 + wr[key] * 1024
        r = {"kernel": name, "grid": grid, "FETCH_SIZE_KB_median": fe[key], "WRITE_SIZE_KB_median": wr[key],
             "hbm_bytes_per_launch": int(hbm)}
        rows.append(r)
        print(json.dumps(r))
    if a.out and a.tag_map:
        tags = json.loads(a.tag_map)
        try:
            d = json.load(open(a.out))
        except FileNotFoundError:
            d = {}
        for tag, (sub, grid, alg) in tags.items():
            hit = [r for r in rows if sub in r["kernel"] and r["grid"] == grid]
            if len(hit) != 1:
                print(f"tag {tag}: {len(hit)} matching groups", file=sys.stderr)
                continue
            r = hit[0]
            d[tag] = {"kernel": r["kernel"], "source": a.source, "FETCH_SIZE_KB_median": r["FETCH_SIZE_KB_median"],
                      "WRITE_SIZE_KB_median": r["WRITE_SIZE_KB_median"],
                      "correction": "FETCH_SIZE x2 for 16-B/lane streaming reads on gfx950 (MI355X_MICROARCH.md §HBM); "
                                    "WRITE_SIZE exact",
                      "hbm_bytes_per_launch": r["hbm_bytes_per_launch"], "algorithmic_bytes_per_launch": alg,
                      "traffic_over_algorithmic": round(r["hbm_bytes_per_launch"] / alg, 6)}
        json.dump(d, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
