import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv)>2 else 16]:
    print(f"{float(r['TotalDurationNs'])/1e6:10.1f} ms {float(r['Percentage']):6.2f}% n={r['Calls']:>6} avg={float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:80]}")
print('total ms', tot/1e6)
