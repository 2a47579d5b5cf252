# LDS bank-conflict model of the wino8 transform jobs (reads b32 and writes b32)
import itertools
def cfg(K, D):
    NCH=(K+3)//4; PAD=D*(K-1)//2; XROWS=64+(NCH-1)*D; ROFF=(4-PAD%4)%4
    RSPAN=(XROWS-1)%D+4*D*((XROWS-1)//D)+6*D+ROFF+1; RSPAN4=(RSPAN+3)//4*4
    RPITCH=RSPAN4 if RSPAN4%8==4 else RSPAN4+4
    return dict(NCH=NCH,PAD=PAD,XROWS=XROWS,ROFF=ROFF,RPITCH=RPITCH,UNITS=XROWS*4)
def conflicts_b32(addrs_by_lane):  # addrs in dwords; groups of 32 lanes; returns extra cycles
    extra=0
    for g in (range(0,32),range(32,64)):
        banks={}
        for l in g:
            a=addrs_by_lane.get(l)
            if a is None: continue
            banks.setdefault(a%32,set()).add(a)
        if banks: extra+=max(len(v) for v in banks.values())-1
    return extra
def sim(K,D,word=lambda uq,pp: 2*uq+pp, ROWB=80):
    c=cfg(K,D); tot_r=tot_w=0; n_r=n_w=0
    for wave in range(4):  # grp0 dense mapping
        units={l:(wave*64+l) for l in range(64)}
        for j in range(4):
            for k in range(7):
                ad={}
                for l,u in units.items():
                    if u>=c['UNITS']: continue
                    urow,uq=u>>2,u&3; ujj,urho=urow//D,urow%D
                    uri=urho+4*D*ujj+c['ROFF']
                    ad[l]=(4*uq+j)*c['RPITCH']+uri+D*k
                tot_r+=conflicts_b32(ad); n_r+=1
        for pp in range(2):
            for p in range(7):
                for q in range(2):
                    ad={}
                    for l,u in units.items():
                        if u>=c['UNITS']: continue
                        urow,uq=u>>2,u&3
                        ad[l]=(p*c['XROWS']*ROWB+urow*ROWB+32*q+4*word(uq,pp))//4
                    tot_w+=conflicts_b32(ad); n_w+=1
    return c, tot_r/n_r, tot_w/n_w
for K in (7,11):
    for D in (1,3,5):
        c,r,w=sim(K,D)
        _,r2,w2=sim(K,D,word=lambda uq,pp: uq+4*pp)
        print(K,D,c['RPITCH'],c['ROFF'],'read extra/instr %.2f'%r,'write %.2f'%w,'-> new word map write %.2f'%w2)


# --- de-interleaved raw rows for D > 1 (wino8_kernel.hpp DEINT): b128 job reads, 16-lane groups
G = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27], [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
G = G + [[l + 32 for l in g] for g in G]


def deint_cost(K, D, RP, CP):
    NCH = (K + 3) // 4
    XROWS = 64 + (NCH - 1) * D
    UNITS = XROWS * 4
    tot = 0
    for wave in range(4):
        for j in range(4):
            for k4 in range(2):
                for g in G:
                    slots = {}
                    for l in g:
                        u = wave * 64 + l
                        if u >= UNITS:
                            continue
                        urow, uq = u >> 2, u & 3
                        ujj, urho = urow // D, urow % D
                        pos = (4 * uq + j) * CP + urho * RP + ujj + k4
                        slots.setdefault(pos % 16, set()).add(pos)
                    if slots:
                        tot += max(len(v) for v in slots.values()) - 1
    return tot


for K in (7, 11):
    for D, RP in ((3, 27), (5, 17)):
        print("deint", K, D, "RP", RP, "extra cycles", deint_cost(K, D, RP, D * RP))
