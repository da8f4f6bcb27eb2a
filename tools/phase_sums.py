#!/usr/bin/env python3
"""Kernel time by phase (prep, fit, candidate chain, pooling) over the last step
(after the last k_fill) of a rocprofv3 kernel trace: union and sum per phase,
the largest kernels.  usage: phase_sums.py KERNEL_TRACE.csv"""
import csv,re,collections,sys
rows=[]
for r in csv.DictReader(open(sys.argv[1])):
    m=re.search(r"(k_\w+)", r["Kernel_Name"]); n=m.group(1) if m else r["Kernel_Name"][:24]
    rows.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),n))
rows.sort()
fills=[r for r in rows if r[2]=='k_fill']
t0=fills[-1][0]
sel=[r for r in rows if r[0]>=t0]
def union(iv):
    tot=0; cs=ce=None
    for s,e in sorted(iv):
        if cs is None or s>ce:
            if cs is not None: tot+=ce-cs
            cs,ce=s,e
        else: ce=max(ce,e)
    if cs is not None: tot+=ce-cs
    return tot/1e6
cls=collections.defaultdict(list)
for s,e,n in sel:
    c='fit' if n.startswith('k_fit') else 'pool' if n in('k_pool2','k_pool','k_pool_ovf') else 'chain' if n in ('k_cand','k_cand_export','k_flow','k_pool_compact','k_true_polar','k_import_flows','k_export_flows','k_cand_list','k_cand_commit') else 'prep'
    cls[c].append((s,e))
span=(max(r[1] for r in sel)-t0)/1e6
print(f"span {span:.1f} ms, any {union([(s,e) for s,e,_ in sel]):.1f}")
for c,iv in cls.items(): print(f"  {c:6s} union {union(iv):7.2f} ms  sum {sum(e-s for s,e in iv)/1e6:7.2f} ms  n={len(iv)}")
k=collections.defaultdict(list)
for s,e,n in sel: k[n].append((s,e))
for n,iv in sorted(k.items(), key=lambda kv:-sum(e-s for s,e in kv[1]))[:14]:
    print(f"    {n:26s} n={len(iv):5d} sum {sum(e-s for s,e in iv)/1e6:7.2f} union {union(iv):7.2f}")
