"""Constant-rate model of the batch kernel's stream queue (config 2): 4096 streams whose rolled
work is min(Exp(4 MiB), 2 MiB) (the first candidate after the 2 MiB minimum, else the stream end),
2048 waves, FIFO visits of at most Q scanned bytes.  Prints the makespan over the perfectly
balanced one.  Not a measurement: DESIGN.md §5 compares it with the measured quantum A/B (the
model has no hand-off cost and keeps every wave's rate constant)."""
import heapq, numpy as np
rng=np.random.default_rng(1)
M=1<<20
def sim(ns=4096, nw=2048, Q=768*1024, order='fifo', reps=5):
    res=[]
    for r in range(reps):
        W=np.minimum(rng.exponential(4*M, ns), 2*M)
        rem=list(W); queue=list(range(ns))
        if order=='lpt': queue.sort(key=lambda i:-rem[i])
        from collections import deque
        q=deque(queue); ev=[]; t=0.0
        busy=0.0
        for w in range(nw):
            if q: s=q.popleft(); d=min(Q, rem[s]); rem[s]-=d; heapq.heappush(ev,(d,w,s))
        end=0
        while ev:
            t,w,s=heapq.heappop(ev); end=max(end,t)
            if rem[s]>1e-9: q.append(s)
            if q:
                s2=q.popleft(); d=min(Q if len(q)>0 else 1e18, rem[s2]) if True else 0
                d=min(Q, rem[s2]); rem[s2]-=d; heapq.heappush(ev,(t+d,w,s2))
        ideal=W.sum()/nw
        res.append(end/ideal)
    return np.mean(res)
for Q in [256*1024, 768*1024, 2*M]:
    print(Q>>10, 'KiB fifo makespan/ideal', round(sim(Q=Q),3))
for Q in [128*1024, 384*1024, 512*1024]:
    print(Q>>10, 'KiB fifo makespan/ideal', round(sim(Q=Q),3))
