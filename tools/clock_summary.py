"""Shader clock held under k_zline per library variant (tools/gpu_clock_ab.sh output):
GRBM_GUI_ACTIVE counts the dispatch's GPU-busy cycles summed over the 8 XCDs (bench.py
clock_GHz); over the dispatch's duration that is the clock.  Usage: python tools/clock_summary.py <dir> v1 v2 ..."""
import csv
import glob
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    d, vs = sys.argv[1], sys.argv[2:]
    for v in vs:
        ctr = rows(f"{d}/{v}/**/*counter_collection.csv")
        gui, dur = {}, {}
        for r in ctr:
            if "k_zline" in r.get("Kernel_Name", "") and r.get("Counter_Name") == "GRBM_GUI_ACTIVE":
                gui[r["Dispatch_Id"]] = float(r["Counter_Value"]) / 8.0
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        ids = [i for i in gui if i in dur]
        if not ids:
            print(v, "no k_zline dispatches with both counter and trace rows")
            continue
        clk = [gui[i] / dur[i] / 1e9 for i in ids]
        ms = [dur[i] * 1e3 for i in ids]
        print(f"{v}: {len(ids)} dispatches, clock {min(clk):.3f}-{max(clk):.3f} GHz "
              f"(mean {sum(clk) / len(clk):.3f}), {sum(ms) / len(ms):.3f} ms per dispatch")


if __name__ == "__main__":
    main()
