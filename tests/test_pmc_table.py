"""tools/pmc_table.py on synthetic rocprofv3 CSVs (no GPU): counters summed per kernel, derived columns."""
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))

import pmc_table  # noqa: E402


def _write(d, counters, trace):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "p_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writerows(counters)
    with open(os.path.join(d, "p_kernel_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerows(trace)


def test_pmc_table(tmp_path):
    trace = [["gemm", 0, 1_000_000], ["gemm", 2_000_000, 3_000_000], ["bn", 0, 1_000_000]]
    _write(tmp_path / "sq", [
        [1, "gemm", "GRBM_GUI_ACTIVE", 8 * 1000], [1, "gemm", "SQ_VALU_MFMA_BUSY_CYCLES", 256 * 500],
        [2, "gemm", "GRBM_GUI_ACTIVE", 8 * 1000], [2, "gemm", "SQ_VALU_MFMA_BUSY_CYCLES", 256 * 500],
        [1, "gemm", "SQ_INSTS_LDS", 100], [1, "gemm", "SQ_LDS_BANK_CONFLICT", 50],
        [3, "bn", "GRBM_GUI_ACTIVE", 8000]], trace)
    _write(tmp_path / "fe", [[3, "bn", "FETCH_SIZE", 1e6]], trace)
    _write(tmp_path / "wr", [[3, "bn", "WRITE_SIZE", 1e6]], trace)
    out = tmp_path / "t.md"
    pmc_table.main(str(tmp_path / "sq"), str(tmp_path / "fe"), str(tmp_path / "wr"), 5, str(out))
    rows = {l.split("`")[1]: l for l in out.read_text().splitlines() if l.startswith("| ") and "`" in l}
    g = [c.strip() for c in rows["gemm"].split("|")]
    assert g[1] == "2.00" and g[3] == "2" and g[4] == "0.50" and g[5] == "0.50"
    b = [c.strip() for c in rows["bn"].split("|")]
    assert b[6] == "3,072"  # (2 * 1e6 + 1e6) KiB over 1 ms
