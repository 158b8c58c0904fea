#!/usr/bin/env python3
"""Same-run comparison of a tune.py JSON against a table: for every op, the table choice's time
vs the best candidate whose config matches a regex.  tools/tune_cmp.py tune.json old.tune REGEX [N]"""
import json,re,collections,sys
d=json.load(open(sys.argv[1]))['results']
prev={}
for l in open(sys.argv[2]):
    m=re.match(r"(.*) cfg=(\S+) splits=(\d+) red=(\w)", l)
    if m: prev[m.group(1)]=(m.group(2), int(m.group(3))*(-1 if m.group(4)=='k' else 1))
pref=sys.argv[3]
by=collections.defaultdict(list)
for r in d: by[r['key']].append(r)
tot_old=tot_new=0; rows=[]
for k,rs in by.items():
    p=prev.get(k)
    pt=[r['ms'] for r in rs if p and r['cfg']==p[0] and r['splits']==p[1]]
    cand=[r for r in rs if re.match(pref, r['cfg'])]
    if not cand or not pt: continue
    b=min(cand,key=lambda r:r['ms'])
    tot_old+=pt[0]; tot_new+=min(pt[0],b['ms'])
    rows.append((pt[0]-b['ms'], k, p, pt[0]*1e3, b['cfg'], b['splits'], b['ms']*1e3))
rows.sort(reverse=True)
print(len(rows),'ops; table %.4f -> %.4f ms'%(tot_old,tot_new))
for r in rows[:int(sys.argv[4]) if len(sys.argv)>4 else 25]: print('%+.2f'%(r[0]*1e3), r[1], r[2], '%.2f'%r[3], r[4], r[5], '%.2f'%r[6])
