# Bank model of conv3 forward's compact-row tap reads (ds_read_b128 lane groups of MI355X_MICROARCH.md
# §LDS): summed max slot multiplicity per group for pixel-row strides R (16-B units) and chunk swizzles.
#   python tools/conv3_bank_model.py [--search]   (ideal: 216 = every group conflict-free; shipped: R = 10, no
#   swizzle, 432 = 2-way at most; before: R = 8 with c ^ ((p >> 1) & 7), 584)
import random
GROUPS=[list(range(0,4))+list(range(12,16))+list(range(20,28)),
        list(range(4,12))+list(range(16,20))+list(range(28,32)),
        list(range(32,36))+list(range(44,48))+list(range(52,60)),
        list(range(36,44))+list(range(48,52))+list(range(60,64))]
acc=[]
for mt in range(3):
    for kh in range(2):
        for s in range(9):
            ks=9*kh+s; tap=ks>>1; ky,kx=tap//3,tap%3
            for G in GROUPS:
                L=[]
                for lane in G:
                    i16=lane&15; g=lane>>4
                    m=16*mt+i16; p0=9*(m//7)+m%7
                    L.append((p0+9*ky+kx, 4*(ks&1)+g))
                acc.append(L)
def cost(R,f):
    tot=0; worst=0
    for L in acc:
        cnt={}
        for p,c in L:
            sl=(R*p+(c^f[p]))%16
            cnt[sl]=cnt.get(sl,0)+1
        mx=max(cnt.values()); tot+=mx; worst=max(worst,mx)
    return tot,worst
for R in range(8,17):
    f0=[0]*84
    print(R, 'f=0', cost(R,f0), 'f=(p>>1)&7', cost(R,[(p>>1)&7 for p in range(84)]))
import sys
random.seed(7)
for R in ((9, 10, 11, 13, 14) if '--search' in sys.argv else ()):
    best=[0]*84; bc=cost(R,best)
    for it in range(15000):
        f=best[:]
        for _ in range(random.randint(1,3)):
            f[random.randrange(84)]=random.randrange(8)
        c=cost(R,f)
        if c<=bc:
            best,bc=f,c
    print('R',R,'search',bc, best if bc[0]<=260 else '')
