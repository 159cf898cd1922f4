import csv, sys, collections
d = sys.argv[1]
rows = list(csv.DictReader(open(f'{d}/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    nm = r['Name'].replace('void (anonymous namespace)::', '').replace('(anonymous namespace)::', '')
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['Percentage']):5.1f}% n={r['Calls']:>4} avg={float(r['AverageNs'])/1e3:8.1f}us {nm[:90]}")
print('total ms', tot / 1e6)
