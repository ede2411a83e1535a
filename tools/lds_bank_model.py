#!/usr/bin/env python3
"""LDS bank-conflict model of conv_bwd_kernel access patterns (32 banks x 4 B, each 32-lane half of a
wave serviced separately; cycles = max distinct addresses per bank).  Used to pick the padded
strides F_A1R/F_A1C/F_Z1R/F_XR; rerun after touching those layouts."""
# bank-conflict model: per wave instruction, lanes split in halves of 32; cycles = max over banks of #distinct addrs
from collections import defaultdict
def cyc(addrs):
    tot=0
    for h in (addrs[:32], addrs[32:]):
        banks=defaultdict(set)
        for a in h:
            if a is None: continue
            banks[a%32].add(a)
        tot+=max((len(v) for v in banks.values()), default=0)
    return tot  # ideal = 2
F_DS,F_D8,F_WS,F_DC,F_Z1=66,80,144,68,580
res=defaultdict(lambda:[0,0])
def acc(name, addrs):
    c=cyc(addrs); res[name][0]+=c; res[name][1]+=2
for wv in range(8):
  lanes=range(64)
  # phase 2a
  pt=wv&3; jt0=(wv>>2)*4
  for s in range(13):
    acc('2a bv dz80', [(4*s+(l>>4))*F_D8+pt*16+(l&15) for l in lanes])
    for n in range(4):
      acc('2a av w_s', [(4*s+(l>>4))*F_WS+(jt0+n)*16+(l&15) for l in lanes])
  for n in range(4):
    for r in range(4):
      acc('2a C store dcol', [((jt0+n)*16+(l>>4)*4+r)*F_DC+pt*16+(l&15) for l in lanes])
  # phase 2b
  mt=wv&3; nt0=(wv>>2)*4
  for s in range(16):
    acc('2b av dz_s', [(mt*16+(l&15))*F_DS+4*s+(l>>4) for l in lanes])
    poffs=[(s>>1)*12+4*(s&1)+(l>>4) for l in lanes]
    for n in range(4):
      ad=[]
      for l in lanes:
        j=(nt0+n)*16+(l&15); jc=min(j,124); ci=jc//25; t=jc-ci*25
        ad.append(ci*144+(t//5)*12+(t%5)+poffs[l] if j<125 else None)
      acc('2b bv a1_s', ad)
# phase 3 (threads 0..719, 2 per thread): reads dcol, writes dz1
for k in range(2):
  for w in range(8):
    es=[w*64+l+k*512 for l in range(64)]
    for kh in range(5):
      for kw in range(5):
        ad=[]
        for e in es:
          if e>=720: ad.append(None); continue
          c=e//144; p=e-c*144; y=p//12; x=p-y*12; oy=y-kh; ox=x-kw
          ok=0<=oy<=7 and 0<=ox<=7
          ad.append((c*25+kh*5+kw)*F_DC+oy*8+ox if ok else 0)
        acc('3 dcol read', ad)
    for dd in (0,1,24,25):
      ad=[]
      for e in es:
        if e>=720: ad.append(None); continue
        c=e//144; p=e-c*144; y=p//12; x=p-y*12
        ad.append(c*F_Z1+(2*y)*24+2*x+dd)
      acc('3 dz1 store', ad)
# phase 4 VALU: threads<400
for w in range(7):
  tids=[w*64+l for l in range(64)]
  for yy in range(3):
    for q in range(16):
      ad=[]
      for t in tids:
        if t>=400: ad.append(None); continue
        c=t//80; rem=t-c*80; kh=rem>>4; part=rem&15; ry=part>>1; cx=(part&1)*12
        ad.append(784*0 + (ry*3+yy+kh)*28+cx+q)
      acc('4 x_s read', ad)
    for x in range(12):
      ad=[]
      for t in tids:
        if t>=400: ad.append(None); continue
        c=t//80; rem=t-c*80; part=rem&15; ry=part>>1; cx=(part&1)*12
        ad.append(c*F_Z1+(ry*3+yy)*24+cx+x)
      acc('4 dz1 read', ad)
tot=0
for k,(c,i) in sorted(res.items(), key=lambda kv:-(kv[1][0]-kv[1][1])):
    print(f"{k:18s} cycles={c:6d} ideal={i:6d} excess={c-i:6d}")
    tot+=c-i
print('total excess per block', tot)
