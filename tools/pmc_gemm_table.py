"""Derived per-kernel metrics of the GEMM PMC passes (tools/pmc_gemm.sh + tools/pmc_gemm2.sh, same tag):
where a persistent GEMM's cycles go -- MFMA pipe, LDS instruction issue, vector-memory (LDS-DMA)
issue and in-flight depth, texture-address (TA) / data (TD) pipe occupancy and the L2 read latency.
Units: GRBM_GUI_ACTIVE / 8 = kernel cycles per XCD (MI355X_MICROARCH.md), SQ_* quad-cycle counters x 4,
per-CU counters (TA/TD/TCP _sum) divided by 256 CUs.
usage: python tools/pmc_gemm_table.py gpurun_out <tag> [<tag> ...] [--all: non-MFMA kernels too]"""
import collections
import csv
import glob
import re
import sys


def load(root, tag):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in (f"{root}/pmc_{tag}", f"{root}/pmc2_{tag}"):
        for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
                    k = re.sub(r"\(.*$", "", k).replace("void ", "").replace("cg::", "").strip()
                    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    allk = "--all" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--all"]
    root, tags = args[0], args[1:]
    for tag in tags:
        acc = load(root, tag)
        for k, c in acc.items():
            m = lambda n: (sum(c[n]) / len(c[n])) if c.get(n) else float("nan")  # noqa: E731
            if not allk and (not c.get("SQ_INSTS_MFMA") or m("SQ_INSTS_MFMA") == 0):
                continue
            if not c.get("GRBM_GUI_ACTIVE"):
                continue
            gui = m("GRBM_GUI_ACTIVE") / 8            # kernel cycles (per XCD)
            simd = gui * 1024                          # SIMD-cycles over the chip
            cu = gui * 256                             # CU-cycles over the chip
            rows = [
                ("MFMA busy (of SIMD cycles)", m("SQ_VALU_MFMA_BUSY_CYCLES") / simd),
                ("VALU+MFMA co-exec", m("SQ_VALU_MFMA_COEXEC_CYCLES") / simd),
                ("LDS instr. active (SQ_ACTIVE_INST_LDS x4)", 4 * m("SQ_ACTIVE_INST_LDS") / simd),
                ("LDS pipe busy (SQ_LDS_IDX_ACTIVE x4 / CU cycles)", 4 * m("SQ_LDS_IDX_ACTIVE") / cu),
                ("VMEM instr. active (SQ_ACTIVE_INST_VMEM x4)", 4 * m("SQ_ACTIVE_INST_VMEM") / simd),
                ("TA busy (TA_BUSY_avr / kernel cycles)", m("TA_BUSY_avr") / gui),
                ("TA addr stalled by TC (per CU)", m("TA_ADDR_STALLED_BY_TC_CYCLES_sum") / cu),
                ("TD busy (per CU)", m("TD_TD_BUSY_sum") / cu),
                ("TD stalled by TC (per CU)", m("TD_TC_STALL_sum") / cu),
                ("TCP pending stall (per CU)", m("TCP_PENDING_STALL_CYCLES_sum") / cu),
                ("SQ->TA addr FIFO full (x4 / SIMD cycles)", 4 * m("SQ_VMEM_TA_ADDR_FIFO_FULL") / simd),
                ("LDS data FIFO full (x4 / SIMD cycles)", 4 * m("SQ_LDS_DATA_FIFO_FULL") / simd),
                ("waves parked: s_waitcnt / barrier (SQ_WAIT_ANY)", m("SQ_WAIT_ANY") / m("SQ_WAVE_CYCLES")),
                ("issue stalls: dependency / pipe (SQ_WAIT_INST_ANY)", m("SQ_WAIT_INST_ANY") / m("SQ_WAVE_CYCLES")),
            ]
            print(f"== {tag}: {k[:70]}  ({len(c.get('SQ_INSTS_MFMA', []))} launches, "
                  f"{gui / 2.1e3:.1f} us at 2.1 GHz)")
            for name, v in rows:
                print(f"   {name:52s} {100 * v:6.1f} %")
            lat = m("TCP_TCC_READ_REQ_LATENCY_sum") / max(1.0, m("TCP_TCC_READ_REQ_sum"))
            lvl = m("SQ_INST_LEVEL_VMEM") / max(1.0, m("SQ_INSTS_VMEM"))
            print(f"   {'L2 read latency (TCP->TCC, cycles)':52s} {lat:8.0f}")
            print(f"   {'VMEM instr. in flight per instr. (INST_LEVEL/INSTS)':52s} {lvl:8.0f}")
            print(f"   instructions per launch: MFMA {m('SQ_INSTS_MFMA') / 1e6:.2f} M, LDS {m('SQ_INSTS_LDS') / 1e6:.2f} M, "
                  f"VMEM {m('SQ_INSTS_VMEM') / 1e6:.2f} M, VALU {m('SQ_INSTS_VALU') / 1e6:.2f} M, "
                  f"SALU {m('SQ_INSTS_SALU') / 1e6:.2f} M")
            hit, miss = m("TCC_HIT_sum"), m("TCC_MISS_sum")
            print(f"   HBM read {2 * m('FETCH_SIZE') / 1024:.1f} MB (FETCH_SIZE x2), write {m('WRITE_SIZE') / 1024:.1f} MB, "
                  f"L2 hit {100 * hit / max(1.0, hit + miss):.1f} %")


if __name__ == "__main__":
    main()
