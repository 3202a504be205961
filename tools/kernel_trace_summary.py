import csv, collections, sys
for d in sys.argv[1:]:
    rows=list(csv.DictReader(open(d)))
    agg=collections.defaultdict(list)
    for r in rows:
        n=r["Kernel_Name"]
        if "at::native" in n or "copyBuffer" in n or "pack" in n: continue
        short=n.split("(anonymous namespace)::")[1].split("(")[0]
        g=(r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z"))
        agg[(short,g)].append(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))
    print("==",d)
    for k,v in sorted(agg.items(), key=lambda kv:-sum(kv[1])):
        v=sorted(v); print(f"  {k[0]:40s} grid={k[1]} n={len(v)} med={v[len(v)//2]/1e3:.1f}us")
