#!/usr/bin/env python3
"""Per-millisecond busy time of the fit, pooling and chain kernels over the last
step (after the last k_fill) of a rocprofv3 kernel trace: do the sweeps overlap?
usage: fit_pool_overlap.py KERNEL_TRACE.csv"""
import csv,re,collections,sys
rows=[]
for r in csv.DictReader(open(sys.argv[1])):
    m=re.search(r"(k_\w+)", r["Kernel_Name"]); n=m.group(1) if m else r["Kernel_Name"][:20]
    rows.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),n,r["Queue_Id"]))
rows.sort()
fills=[r for r in rows if r[2]=='k_fill']
t0=fills[-1][0]
sel=[r for r in rows if r[0]>=t0]
span=(max(r[1] for r in sel)-t0)/1e6
bins=collections.defaultdict(lambda: collections.Counter())
for s,e,n,q in sel:
    cls='fit' if n.startswith('k_fit') else 'pool' if n in('k_pool2','k_pool','k_pool_ovf') else 'chain'
    b0=int((s-t0)//1e6); b1=int((e-t0)//1e6)
    for b in range(b0,b1+1):
        lo=max(s,t0+b*1e6); hi=min(e,t0+(b+1)*1e6)
        if hi>lo: bins[b][cls]+= (hi-lo)/1e3
both=sum(1 for b in bins if bins[b]['fit']>200 and bins[b]['pool']>200)
print(f"step span {span:.1f} ms; 1-ms bins with both fit and pool > 0.2 ms: {both} of {len(bins)}")
for b in sorted(bins)[:40]:
    c=bins[b]; print(f"{b:4d} ms: fit {c['fit']:7.0f}us pool {c['pool']:7.0f}us chain {c['chain']:6.0f}us")
