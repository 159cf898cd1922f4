"""Per-step kernel table from a rocprofv3 kernel trace: the kernels between the last two
optimizer launches, aggregated by (name, grid).
    python tools/step_kernels.py <trace.csv> [top]"""
import collections
import csv
import sys


def main(path, top=40):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows)
           if "adam" in r["Kernel_Name"].lower() or "multi_tensor_apply" in r["Kernel_Name"]]
    last = opt[-1]
    prev = [i for i in opt if i < last - 50][-1]
    step = rows[prev + 1:last + 1]
    agg = collections.OrderedDict()
    tot = 0.0
    for r in step:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        tot += dur
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        n = n.split("(")[0]
        key = (n, r["Grid_Size_X"])
        agg.setdefault(key, [0, 0.0])
        agg[key][0] += 1
        agg[key][1] += dur
    print(f"step kernels {len(step)}, sum {tot:.1f} us")
    for (n, gx), (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{d:9.1f} {c:3d} {gx:>9} {n[:100]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
