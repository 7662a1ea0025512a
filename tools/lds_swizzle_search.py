import itertools
G=[list(range(0,4))+list(range(12,16))+list(range(20,28)),
   list(range(4,12))+list(range(16,20))+list(range(28,32))]
G+= [[x+32 for x in g] for g in G]
def ok(f):
    for g in G:
        s=set()
        for l in g:
            row=l&15; kq=l>>4
            s.add((row*4 + (kq ^ f(row)))%16)
        if len(s)!=16: return False
    return True
cands={'r>>2':lambda r:(r>>2)&3,'(r>>1)&3':lambda r:(r>>1)&3,'r&3':lambda r:r&3,
 'r>>2 ^ r&3':lambda r:((r>>2)^r)&3}
for n,f in cands.items(): print(n, ok(f))
# brute force table over row 0..15
sols=0
for tab in itertools.product(range(4),repeat=4):
    f=lambda r,t=tab: t[(r>>2)&3]
    if ok(f): print('tab by r>>2',tab); sols+=1
for tab in itertools.product(range(4),repeat=4):
    f=lambda r,t=tab: t[r&3]
    if ok(f): print('tab by r&3',tab); break
print("BK64")
def ok64(f):
    for s in range(2):
      for g in G:
        sl=set()
        for l in g:
            row=l&15; ch=4*s+(l>>4)
            sl.add((row*8 + (ch ^ f(row)))%16)
        if len(sl)!=16: return False
    return True
for n,f in {'(r>>1)&7':lambda r:(r>>1)&7,'r&7':lambda r:r&7,'(r>>1)&3':lambda r:(r>>1)&3, '((r>>1)&3)<<1|r&1': lambda r: (((r>>1)&3)<<1)|(r&1), 'r>>1 &7 ^ ...':lambda r:((r>>1)&7)}.items(): print(n, ok64(f))
