"""Python model of k_bpe_long's LDS path (tokenize_bpe.hip, r04): merge values cached per pair,
carried through the in-place compaction, invalidated next to merged symbols and re-probed, against
the uncached loop (every pair probed every step).  Wave semantics are modelled tile by tile (64
lanes in lockstep).  tests/test_bpe_long_model.py runs it on random merge tables."""
import random
def lma(m, blocked):
    sel=0
    if blocked: m &= ~1
    while m:
        s = m & ~(m<<1) & ((1<<64)-1)
        sel |= s
        m &= ~(s | (s<<1))
    return sel
def popc(x): return bin(x).count('1')
def ref(sym, mv):
    m=len(sym); sym=list(sym)
    while True:
        rmin=0xFFFF
        for j in range(m-1):
            r=mv(sym[j],sym[j+1])>>16; rmin=min(rmin,r)
        if rmin==0xFFFF: break
        out=[]; blocked=False
        for t0 in range(0,m,64):
            vals=[]; cand=0
            for lane in range(64):
                j=t0+lane
                if j+1<m:
                    v=mv(sym[j],sym[j+1])
                    if (v>>16)==rmin: cand|=1<<lane
            sel=lma(cand,blocked)
            tile=((1<<64)-1) if m-t0>=64 else (1<<(m-t0))-1
            live=tile & ~(sel<<1)
            if blocked: live&=~1
            for lane in range(64):
                j=t0+lane
                if (live>>lane)&1:
                    me=(sel>>lane)&1
                    out.append(mv(sym[j],sym[j+1])&0xFFFF if me else sym[j])
            blocked=bool((sel>>63)&1)
        sym=out; m=len(sym)
    return sym
def new(sym, mv):
    NOVAL=0xFFFFFFFE
    n=len(sym); sym=list(sym)+[0]*65; val=[None]*(n+65)
    for j in range(n-1): val[j]=mv(sym[j],sym[j+1])
    mm=n
    while True:
        rmin=0xFFFF
        for j in range(mm-1): rmin=min(rmin,val[j]>>16)
        if rmin==0xFFFF: break
        blocked=False; outp=0
        for t0 in range(0,mm,64):
            S=[sym[t0+l] if t0+l<mm else 0 for l in range(64)]
            V=[val[t0+l] if t0+l+1<mm else 0xFFFFFFFF for l in range(64)]
            cand=0
            for l in range(64):
                if t0+l+1<mm and (V[l]>>16)==rmin: cand|=1<<l
            sel=lma(cand,blocked)
            tile=((1<<64)-1) if mm-t0>=64 else (1<<(mm-t0))-1
            live=tile & ~(sel<<1)
            if blocked: live&=~1
            writes=[]
            for l in range(64):
                me=(sel>>l)&1
                nxt=(sel>>(l+1))&1 if l<63 else 0
                out=(V[l]&0xFFFF) if me else S[l]
                outv=NOVAL if (me or nxt) else V[l]
                if (live>>l)&1:
                    o=outp+popc(live & ((1<<l)-1))
                    writes.append((o,out,outv))
            for o,a,b in writes: sym[o]=a; val[o]=b
            outp+=popc(live); blocked=bool((sel>>63)&1)
        mm=outp
        # left-neighbour pass (lockstep per tile)
        for t0 in range(0,mm,64):
            snap=[(val[j+1], val[j]) if j+1<mm else None for j in range(t0,t0+64)]
            for i,j in enumerate(range(t0,t0+64)):
                if j+1<mm:
                    a,b=snap[i]
                    if a==NOVAL and b not in (NOVAL,0xFFFFFFFD): val[j]=0xFFFFFFFD
        if mm>0: val[mm-1]=0xFFFFFFFF
        for j in range(mm-1):
            if val[j] in (NOVAL, 0xFFFFFFFD): val[j]=mv(sym[j],sym[j+1])
    return sym[:mm]
def run(trials, seed=1):
  random.seed(seed)
  for trial in range(trials):
      A=random.randint(2,6)
      table={}
      nsym=A
      ranks=list(range(1,400)); random.shuffle(ranks)
      ri=0
      for _ in range(random.randint(5,60)):
          a=random.randrange(nsym); b=random.randrange(nsym)
          if (a,b) in table: continue
          table[(a,b)]=(ranks[ri]<<16)|nsym; ri+=1; nsym+=1
      mv=lambda a,b: table.get((a,b),0xFFFFFFFF)
      L=random.randint(2,300)
      s=[random.randrange(A) for _ in range(L)]
      r=ref(s,mv); x=new(s,mv)
      if r!=x:
          raise AssertionError(('mismatch', trial, L))
  return True



if __name__ == '__main__':
    print(run(20000))
