#!/usr/bin/env python3
"""Per-kernel PMC digest table (markdown) from a tools/pmc_summary.py text file.

Columns: waves; MFMA / VALU (incl. MFMA) / LDS instructions per wave; LDS bank-conflict cycles
per dispatch and as a share of LDS-array cycles (SQ_LDS_IDX_ACTIVE); VMEM reads per wave;
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES over the dispatch's SIMD-cycles (GRBM_GUI_ACTIVE is summed
over the 8 XCDs: SIMD-cycles = GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs); and where the waves'
cycles went (SQ_ACTIVE_INST_ANY / SQ_WAIT_INST_ANY / SQ_WAIT_ANY over SQ_WAVE_CYCLES)."""
import re
import sys


def parse(path):
    k, out = None, {}
    for line in open(path):
        m = re.match(r"== (.*)", line)
        if m:
            k = m.group(1).strip()
            out[k] = {}
            continue
        p = line.split()
        if k and len(p) == 2:
            out[k][p[0]] = float(p[1])
    return out


def main(path, want):
    d = parse(path)
    print("| kernel | waves | MFMA/wave | VALU/wave | LDS/wave | LDS bank-conflict cycles (% of LDS cycles) "
          "| VMEM rd/wave | MFMA busy | active / wait-issue / wait-mem of wave cycles |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name in d:
        if want and not any(w in name for w in want):
            continue
        c = d[name]
        wv = c.get("SQ_WAVES", 0)
        if not wv:
            continue
        simd = c.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd if simd else 0
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0)
        print(f"| `{name}` | {wv:.0f} | {c.get('SQ_INSTS_MFMA', 0) / wv:.1f} | {c.get('SQ_INSTS_VALU', 0) / wv:.0f} "
              f"| {c.get('SQ_INSTS_LDS', 0) / wv:.1f} | {bc:.0f} ({100 * bc / lds if lds else 0:.0f} %) "
              f"| {c.get('SQ_INSTS_VMEM_RD', 0) / wv:.1f} | {100 * busy:.1f} % "
              f"| {100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0f} / {100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:.0f} "
              f"/ {100 * c.get('SQ_WAIT_ANY', 0) / wc:.0f} % |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
