import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
n=len(rows); sub=rows[int(n*0.3):int(n*0.7)]
t0=int(sub[0]['Start_Timestamp']); t1=max(int(r['End_Timestamp']) for r in sub)
ev=[]
for r in sub: ev+=[(int(r['Start_Timestamp']),1),(int(r['End_Timestamp']),-1)]
ev.sort(); cur=0; last=t0; hist=collections.Counter()
for t,d in ev:
    hist[cur]+=t-last; last=t; cur+=d
span=t1-t0
print('span us', round(span/1e3,1), 'kernels', len(sub), 'concurrency', {c: round(v/span,3) for c,v in sorted(hist.items())})
print('queues', dict(collections.Counter(r['Queue_Id'] for r in sub)), 'streams/queue',
      {q: len({r['Stream_Id'] for r in sub if r['Queue_Id']==q}) for q in {r['Queue_Id'] for r in sub}})
agg=collections.defaultdict(lambda:[0,0])
for r in sub: agg[r['Kernel_Name'][:34]][0]+=int(r['End_Timestamp'])-int(r['Start_Timestamp']); agg[r['Kernel_Name'][:34]][1]+=1
for k,v in sorted(agg.items(), key=lambda x:-x[1][0]): print(f'  {k:36s} {v[1]:5d} avg {v[0]/v[1]/1e3:7.1f} us')
