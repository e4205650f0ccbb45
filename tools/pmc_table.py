"""Per-kernel-family table of rocprofv3 PMC counters (summed over dispatches)."""
import csv
import sys
from collections import defaultdict

rows = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("mvp::", "")
        name = name.split("(")[0][:44]
        rows[name][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[name].add(r["Dispatch_Id"])
cols = sorted({c for v in rows.values() for c in v})
order = sorted(rows, key=lambda k: -rows[k].get("SQ_WAVE_CYCLES", 0))
for k in order:
    d = rows[k]
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    out = [f"{k:44s} n={len(calls[k]):3d}"]
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if c in d:
            out.append(f"{c.replace('SQ_', '').replace('ACTIVE_INST', 'ACT')}={d[c] / wc:5.2f}")
    if "SQ_LDS_IDX_ACTIVE" in d:
        out.append(f"LDSconf={d.get('SQ_LDS_BANK_CONFLICT', 0) / max(d['SQ_LDS_IDX_ACTIVE'], 1):5.2f}")
    if "SQ_INSTS_MFMA" in d and "SQ_WAVES" in d:
        out.append(f"mfma/wave={d['SQ_INSTS_MFMA'] / max(d['SQ_WAVES'], 1):7.0f}")
    if "SQ_INSTS_VALU" in d and "SQ_INSTS_LDS" in d:
        out.append(f"valu={d['SQ_INSTS_VALU']:.3g} lds={d['SQ_INSTS_LDS']:.3g} vmem={d.get('SQ_INSTS_VMEM', 0):.3g}")
    print("  ".join(out))
    extra = []
    if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
        # per-SIMD MFMA busy over the kernel's active cycles, 256 CUs x 4 SIMDs
        extra.append(f"mfma_busy={d['SQ_VALU_MFMA_BUSY_CYCLES'] / max(d['GRBM_GUI_ACTIVE'] * 1024, 1):5.3f}")
    if "FETCH_SIZE" in d:
        extra.append(f"fetchMB/launch={2 * d['FETCH_SIZE'] * 1024 / len(calls[k]) / 1e6:8.1f}")
    if "WRITE_SIZE" in d:
        extra.append(f"writeMB/launch={d['WRITE_SIZE'] * 1024 / len(calls[k]) / 1e6:8.1f}")
    if extra:
        print("    " + "  ".join(extra))
