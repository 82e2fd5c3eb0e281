import csv,sys,statistics
from collections import defaultdict
d=sys.argv[1]
rows=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
ev=[]
for r in rows:
    n=r['Kernel_Name']
    k='hash' if 'chain_step' in n else 'gather' if 'gather' in n else 'split' if 'split_batch' in n else 'blit' if 'copyBuffer' in n else 'other'
    ev.append((int(r['Start_Timestamp']),int(r['End_Timestamp']),k,r['Queue_Id']))
ev.sort()
t0=ev[0][0]
tot=defaultdict(float); cnt=defaultdict(int)
for s,e,k,_ in ev: tot[k]+=(e-s)/1e6; cnt[k]+=1
print({k:(round(v,1),cnt[k]) for k,v in tot.items()}, 'span', (ev[-1][1]-t0)/1e6)
hs=[(s,e) for s,e,k,_ in ev if k=='hash']
gaps=[(hs[i+1][0]-hs[i][1])/1e6 for i in range(len(hs)-1)]
print('hash kernels',len(hs),'mean dur',round(statistics.mean((e-s)/1e6 for s,e in hs),3),'gap mean',round(statistics.mean(gaps),3),'median',round(statistics.median(gaps),3), 'max', round(max(gaps),3))
# what overlaps the biggest gaps
big=sorted(range(len(gaps)),key=lambda i:-gaps[i])[:5]
for i in big:
    a,b=hs[i][1],hs[i+1][0]
    ov=[(k,round((min(e,b)-max(s,a))/1e6,3)) for s,e,k,_ in ev if s<b and e>a and k!='hash']
    print('gap',round(gaps[i],3),'at',round((a-t0)/1e6,1),ov[:8])
mc=list(csv.DictReader(open(d+'/run_memory_copy_trace.csv')))
dd=defaultdict(float);c=defaultdict(int)
for r in mc:
    k=r.get('Direction') or r.get('Kind'); dd[k]+=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6; c[k]+=1
print(dict(dd),dict(c))
