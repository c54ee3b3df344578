"""LDS per workgroup of the DP kernel's dispatches, from a rocprofv3
--kernel-trace CSV, and the waves per SIMD that LDS (160 KB per CU) and the
kernel's VGPRs (512 per SIMD lane) allow.  Dispatch count and kernel time per
(instance, LDS size).

  python tools/lds_occupancy.py run_kernel_trace.csv
"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    cols = rows[0].keys() if rows else []
    lds_col = next((c for c in ("LDS_Block_Size", "Lds_Size", "LDS_Size") if c in cols), None)
    vgpr_col = next((c for c in ("Arch_VGPR_Count", "VGPR_Count") if c in cols), None)
    wg_col = next((c for c in ("Workgroup_Size", "Workgroup_Size_X") if c in cols), None)
    print("columns:", lds_col, vgpr_col, wg_col)
    n = collections.Counter()
    ms = collections.Counter()
    for r in rows:
        name = r["Kernel_Name"]
        if "poa_strip_kernel" not in name:
            continue
        inst = name.split("(")[0].split("poa_strip_kernel")[-1]
        lds = int(r[lds_col]) if lds_col else -1
        vgpr = int(r[vgpr_col]) if vgpr_col else -1
        wg = int(r[wg_col]) if wg_col else -1
        k = (inst, lds, vgpr, wg)
        n[k] += 1
        ms[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    total = sum(ms.values()) or 1.0
    for k in sorted(n, key=lambda x: -ms[x]):
        inst, lds, vgpr, wg = k
        waves_wg = max(1, wg // 64)
        by_lds = (160 * 1024 // lds) * waves_wg / 4 if lds > 0 else float("inf")
        by_vgpr = 512 // max(vgpr, 1) if vgpr > 0 else float("inf")
        print(f"{inst} lds {lds} B vgpr {vgpr} wg {wg}: {n[k]} dispatches, {ms[k]:.1f} ms ({ms[k] / total:.1%}); "
              f"waves/SIMD by LDS {by_lds:.2f}, by VGPR {by_vgpr}")


if __name__ == "__main__":
    main(sys.argv[1])
