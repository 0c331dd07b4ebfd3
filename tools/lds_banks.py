#!/usr/bin/env python
"""LDS bank-conflict model of the 16-channel residual backward kernel's accesses (resblock.hip
res_bwd16_kernel) for candidate halo'd-tile layouts (pixel stride, row stride, image stride),
and (--wgrad) of conv.hip conv_wgrad_kernel's tr reads, plain NHWC vs the swizzled tile.

Lane groups and bank rules per instruction from MI355X_MICROARCH.md section LDS: ds_read_b128
4 x 16 lanes (interleaved groups), 64 banks; ds_read_b64 / ds_read_b64_tr_b16 2 x 32, 64 banks;
ds_write_b64 4 x 16 and ds_write_b128 8 x 8 contiguous lanes, 32 banks. Prints the cycles per
lane group (1.0 = conflict-free) of each access type and a weighted search over layouts.

  python tools/lds_banks.py [--wgrad]
"""
import sys
G128=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128+= [[l+32 for l in g] for g in G128]
G64=[list(range(32)), list(range(32,64))]
GW64=[list(range(i,i+16)) for i in range(0,64,16)]
GW128=[list(range(i,i+8)) for i in range(0,64,8)]
def cycles(addrs, groups, width_words, nbanks):
    tot=0
    for grp in groups:
        banks={}
        for l in grp:
            a=addrs[l]
            if a is None: continue
            for w in range(width_words):
                b=(a//4+w)%nbanks
                banks.setdefault(b,set()).add(a//4+w)
        tot+=max(len(v) for v in banks.values()) if banks else 0
    return tot
def wgrad_model(CIN, COUT, H, W, imgs, new):
    """Mean LDS cycles per lane group of the X-tap and dY tr reads (1.0 = conflict-free)."""
    Hp, Wp, HW = H + 2, W + 2, H * W
    M = imgs * HW
    XPB, DPB = CIN * 2, COUT * 2
    rowpx = 12 if (new and XPB == 32 and W == 8) else Wp
    def sw(yp, xp):
        if not new: return 0
        if W % 16 == 0: return (xp >> 3) & 1
        if W == 8: return yp & 1
        if W == 4: return (yp >> 1) & 1
        return 0
    def xaddr(im, yp, xp, cb):
        s = sw(yp, xp)
        if XPB == 32:
            xs = xp ^ (s << 2) if W % 16 == 0 else xp
            return ((im * Hp + yp) * rowpx + xs) * 32
        return ((im * Hp + yp) * rowpx + xp) * 64 + ((cb ^ s) * 32)
    def daddr(p, mb):
        b = (p >> 3) & 1 if new else 0
        if DPB == 32: return (p ^ (b << 2)) * 32
        return p * 64 + ((mb ^ b) * 32)
    xt = xn = dt = dn = 0
    for kb in range(M // 32):
        for h in range(2):
            for mb in range(COUT // 16):
                ad = [daddr(kb * 32 + 8 * (l >> 4) + 4 * h + ((l & 15) >> 2), mb) + 8 * (l & 3)
                      for l in range(64)]
                dt += cycles(ad, G64, 2, 64); dn += 2
            for t in range(9):
                for cb in range(CIN // 16):
                    ad = []
                    for l in range(64):
                        p = kb * 32 + 8 * (l >> 4) + 4 * h + ((l & 15) >> 2)
                        im, r = divmod(p, HW); y, x = divmod(r, W)
                        ad.append(xaddr(im, y + t // 3, x + t % 3, cb) + 8 * (l & 3))
                    xt += cycles(ad, G64, 2, 64); xn += 2
    return round(xt / xn, 2), round(dt / dn, 2)
if "--wgrad" in sys.argv:
    print("(cin, cout, H, W, imgs): (X taps, dY) cycles per lane group, plain -> swizzled")
    for cfg in [(32, 16, 16, 16, 2), (16, 32, 8, 8, 4), (32, 32, 4, 4, 8), (32, 32, 8, 8, 4),
                (16, 16, 16, 16, 2), (32, 16, 8, 8, 4), (32, 32, 16, 16, 2)]:
        print(cfg, wgrad_model(*cfg, False), "->", wgrad_model(*cfg, True))
    sys.exit(0)
H=W=8; Hp=Wp=10; imgs=4; HW=64
def layout(PIXB,ROWB,IMGB):
    return lambda im,yy,xx: im*IMGB+yy*ROWB+xx*PIXB
def analyze(L):
    M=imgs*HW
    res={}
    # dgrad b128
    tot=0;n=0
    for pb in range(M//16):
        for c in range(5):
            ad=[]
            for lane in range(64):
                g,li=lane>>4,lane&15
                m=pb*16+li; im,r=divmod(m,HW); y,x=divmod(r,W)
                tap=2*c+(g>>1); tap=min(tap,8); ty,tx=divmod(tap,3)
                ad.append(L(im,y+ty,x+tx)+16*(g&1))
            tot+=cycles(ad,G128,4,64); n+=4
    res['dgrad_b128']=tot/n
    # epilogue b64 read at interior
    tot=0;n=0
    for pb in range(M//16):
        ad=[]
        for lane in range(64):
            g,li=lane>>4,lane&15
            m=pb*16+li; im,r=divmod(m,HW); y,x=divmod(r,W)
            ad.append(L(im,y+1,x+1)+8*g)
        tot+=cycles(ad,G64,2,64); n+=2
    res['epi_b64_read']=tot/n
    tot=0;n=0
    for pb in range(M//16):
        ad=[]
        for lane in range(64):
            g,li=lane>>4,lane&15
            m=pb*16+li; im,r=divmod(m,HW); y,x=divmod(r,W)
            ad.append(L(im,y+1,x+1)+8*g)
        tot+=cycles(ad,GW64,2,32); n+=4
    res['epi_b64_write']=tot/n
    # wgrad tr reads: X taps
    tot=0;n=0
    for kb in range(M//32):
        for t in range(9):
            for h in range(2):
                ad=[]
                for lane in range(64):
                    g,li=lane>>4,lane&15
                    p=kb*32+8*g+4*h+(li>>2); im,r=divmod(p,HW); y,x=divmod(r,W)
                    ty,tx=divmod(t,3)
                    ad.append(L(im,y+ty,x+tx)+8*(li&3))
                tot+=cycles(ad,G64,2,64); n+=2
    res['wgrad_tr']=tot/n
    # staging write b128: element e -> pixel e>>1, half e&1
    tot=0;n=0
    for e0 in range(0,2*M,64):
        ad=[]
        for lane in range(64):
            e=e0+lane; q,p=e&1,e>>1; im,r=divmod(p,HW); y,x=divmod(r,W)
            ad.append(L(im,y+1,x+1)+16*q)
        tot+=cycles(ad,GW128,4,32); n+=8
    res['stage_w128']=tot/n
    return res
for name,L in [("cur 48/480",layout(48,480,4800)),("32/512",layout(32,512,5120)),("32/336",layout(32,336,3360)),("64/640",layout(64,640,6400)),("32/512/5136",layout(32,512,5136)),("32/528",layout(32,528,5280))]:
    print(name, {k:round(v,2) for k,v in analyze(L).items()})
print("search")
W8={'dgrad_b128':10*4,'epi_b64_read':3*2,'epi_b64_write':1*4,'wgrad_tr':20*2,'stage_w128':4.5*8}
best=[]
for PIXB in (32,48,64):
    for ROWB in range(PIXB*10, PIXB*10+640, 16):
        for extra in (0,16,32,48,64,128,256):
            L=layout(PIXB,ROWB,ROWB*10+extra)
            r=analyze(L)
            cost=sum(W8[k]*r[k] for k in r)
            best.append((cost,PIXB,ROWB,extra,{k:round(v,2) for k,v in r.items()}))
best.sort(key=lambda t:t[0])
for b in best[:10]: print(b)
print("current", [b for b in best if b[1]==48 and b[2]==480 and b[3]==0][0])
