"""HBM traffic per launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so
bytes = 2·FETCH_SIZE·1024 + WRITE_SIZE·1024.  The backbone "launch" is one
graph forward (stem + every conv/fuse dispatch of that forward).

    python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json]
"""
import csv
import json
import sys
from collections import defaultdict

GROUPS = {"backbone": ("conv_mfma_kernel", "stem_kernel", "stem_mfma_kernel", "fuse_sum_kernel", "fuse_sum_n_kernel", "conv1x1_kernel",
                       "conv1x1_pair_kernel", "bneck_kernel", "basic_block", "tconv_kernel", "tconv16_kernel", "tblock32_kernel",
                       "tblock32s_kernel", "tblock64_kernel", "s2conv_kernel", "stem2_kernel", "trans1_kernel",
                       "head1x1_kernel", "head_fuse_kernel"),
          "moments": ("moments_kernel",),
          "preprocess": ("preprocess_kernel",), "decode": ("decode_kernel",),
          "triangulate": ("triangulate_reference_kernel", "triangulate_all_views_kernel",
                          "triangulate_tol2_kernel")}


def load(path, counter):
    per = defaultdict(lambda: [0.0, 0])
    launches = defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for g, keys in GROUPS.items():
            if any(k in name for k in keys):
                per[g][0] += float(r["Counter_Value"]) * 1024.0
                if g != "backbone" or "stem" in name:  # one stem dispatch per graph forward
                    launches[g] += 1
    return per, launches


def main():
    fetch, n_f = load(sys.argv[1], "FETCH_SIZE")
    write, n_w = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for g in GROUPS:
        n = n_f.get(g, 0)
        if not n:
            continue
        rd = 2.0 * fetch[g][0] / n
        wr = write[g][0] / max(n_w.get(g, 1), 1)
        out[g] = {"launches": n, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                  "hbm_bytes_per_launch": rd + wr}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
