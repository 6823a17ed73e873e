#!/usr/bin/env python3
# DESIGN.md s5 "Pack || GEMM overlap": event simulation of a fused pack+GEMM persistent launch with the rates
# measured by lab/overlap_lab.hip (tile time by concurrent tiles, the probe's 22 % slowdown of tiles beside the
# pack, per-CU pack rates 20/35/60 GB/s).  Pure Python, no GPU.
# crude event simulation of a fused pack+GEMM persistent launch (1 block per CU, dynamic queue)
import heapq, sys
NCU=256
def T_tile(n):  # us per tile when n tiles run concurrently (power-bound), measured points 64:45.5 128:47.7 256:61.2
    if n<=128: return 45.5+ (max(n,64)-64)*(2.2/64)
    return 47.7+(n-128)*(13.5/128)
def run(order, tiles_m, tiles_n, items_per_panel=32, item_bytes=160e3, hbm=6.0e6, rcu=35e3, slow=0.22, dt=0.05):
    # order: list of ('X',i) / ('W',j) / ('T',i,j) ; items per panel expand
    q=[]
    for o in order:
        if o[0] in 'XW':
            q += [(o[0],o[1])]*items_per_panel
        else: q.append(o)
    done={('X',i):0 for i in range(tiles_m)}; done.update({('W',j):0 for j in range(tiles_n)})
    workers=[None]*NCU  # (kind, key, remaining)
    qi=0; t=0.0; finished_tiles=0; ntiles=tiles_m*tiles_n
    while True:
        # assign
        for w in range(NCU):
            if workers[w] is None and qi<len(q):
                o=q[qi]; qi+=1
                if o[0] in 'XW': workers[w]=['P',o,item_bytes]
                else: workers[w]=['T',o,1.0]
        active_p=[w for w in range(NCU) if workers[w] and workers[w][0]=='P']
        run_t=[w for w in range(NCU) if workers[w] and workers[w][0]=='T' and done[('X',workers[w][1][1])]>=items_per_panel and done[('W',workers[w][1][2])]>=items_per_panel]
        if not active_p and not run_t and qi>=len(q) and all(x is None or x[0]!='T' for x in workers): break
        # rates
        if active_p:
            per=min(rcu, hbm/len(active_p))
            frac=per*len(active_p)/hbm
        else: per=0; frac=0
        nt=len(run_t)
        trate=(1.0/T_tile(nt))/(1+slow*frac) if nt else 0
        for w in active_p:
            workers[w][2]-=per*dt
            if workers[w][2]<=0:
                done[workers[w][1]]+=1; workers[w]=None
        for w in run_t:
            workers[w][2]-=trate*dt
            if workers[w][2]<=0:
                workers[w]=None; finished_tiles+=1
        t+=dt
        if finished_tiles==ntiles and qi>=len(q): break
    return t
def pair_order(tm,tn):
    o=[];S=max(tm,tn)
    for s in range(S):
        if s<tm: o.append(('X',s))
        if s<tn: o.append(('W',s))
        for i in range(min(s,tm-1)+1):
            for j in range(min(s,tn-1)+1):
                if max(i,j)==s: o.append(('T',i,j))
    return o
def wfirst(tm,tn):
    o=[('W',j) for j in range(tn)]
    for i in range(tm):
        o.append(('X',i)); o+= [('T',i,j) for j in range(tn)]
    return o
def serial(tm,tn):
    return [('X',i) for i in range(tm)]+[('W',j) for j in range(tn)]+[('T',i,j) for i in range(tm) for j in range(tn)]
for rcu in (20e3,35e3,60e3):
    print("rcu GB/s",rcu/1e3, "serial",round(run(serial(16,16),16,16,rcu=rcu),1),"pair",round(run(pair_order(16,16),16,16,rcu=rcu),1),"wfirst",round(run(wfirst(16,16),16,16,rcu=rcu),1))
print("C4 32x16")
for rcu in (20e3,35e3,60e3):
    print("rcu",rcu/1e3,"serial",round(run(serial(32,16),32,16,rcu=rcu),1),"pair",round(run(pair_order(32,16),32,16,rcu=rcu),1),"wfirst",round(run(wfirst(32,16),32,16,rcu=rcu),1))
