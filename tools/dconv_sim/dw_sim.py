# numpy emulation of DWgradJob (dconv.h): per-block staging, lane bases, MFMA maps, slab writes
import numpy as np
def dw_pad(c, wd):
    best, bd = c, 99
    for p in range(16):
        d = (wd * (c + p)) % 32; e = d - 16 if d > 16 else 16 - d
        if e < bd: bd, best = e, c + p
    return best
def sim(CIN, COUT, KS, H, TMW, B, S, ST=1, VALID=False):
    W = H; KK = KS*KS*CIN; PT = 0 if VALID else (KS-1)//2; PL = PT
    OH = (H-KS)//ST+1 if VALID else H; OW = OH
    TN = COUT//16; WROWS = 4//TN; MPB = TMW*WROWS; MT = (KK+15)//16; TG = (MT+MPB-1)//MPB
    R = 4; RG = (OH+R-1)//R; WPAD = (OW+3)//4*4; KQ = WPAD//4; WP = (WPAD-1)*ST+KS; RIN = (R-1)*ST+KS
    CS = dw_pad(CIN, ST*WP); COS = dw_pad(COUT, WPAD); XSZ = (RIN*WP*CS+3)//4*4
    rs = np.random.RandomState(2)
    X = rs.rand(B, H, W, CIN); dY = rs.randn(B, OH, OW, COUT)
    SL = (KK+1)*COUT
    slab = np.full((S, SL), np.nan)
    NC = B*RG
    for sp in range(S):
        for tg in range(TG):
            c0 = sp*NC//S; c1 = (sp+1)*NC//S
            acc = {}
            dbs = {}
            for w in range(4):
                j = w % TN; wm = w // TN
                lanes = np.arange(64); r = lanes & 15; g = lanes >> 4
                abase = []
                for i in range(TMW):
                    row = np.minimum(16*(tg*MPB + wm + WROWS*i) + r, KK-1)
                    t = row // CIN; ci = row - t*CIN; ky = t // KS; kx = t - ky*KS
                    abase.append(((g*ST+ky)*WP + kx)*CS + ci)
                bbase = g*WPAD*COS + 16*j + r
                a_acc = np.zeros((TMW, 16, 16)); db = np.zeros(64)
                for c in range(c0, c1):
                    b = c // RG; y0 = (c - b*RG)*R
                    Xs = np.full(XSZ, np.nan); Ys = np.full(R*WPAD*COS, np.nan)
                    for item in range(RIN*WP*(CIN//4)):
                        pix, cq = divmod(item, CIN//4); pr, pc = divmod(pix, WP)
                        iy = y0*ST - PT + pr; ix = pc - PL
                        ok = 0 <= iy < H and 0 <= ix < W
                        Xs[pix*CS + 4*cq: pix*CS + 4*cq + 4] = X[b, iy, ix, 4*cq:4*cq+4] if ok else 0
                    for item in range(R*WPAD*(COUT//4)):
                        pix, cq = divmod(item, COUT//4); pr, pc = divmod(pix, WPAD)
                        oy = y0 + pr; ok = oy < OH and pc < OW
                        Ys[pix*COS + 4*cq: pix*COS + 4*cq + 4] = dY[b, oy, pc, 4*cq:4*cq+4] if ok else 0
                    for kq in range(KQ):
                        bv = np.stack([Ys[bbase + (4*kq+s)*COS] for s in range(4)], 1)
                        for i in range(TMW):
                            av = np.stack([Xs[abase[i] + (4*kq+s)*ST*CS] for s in range(4)], 1)
                            for s in range(4):
                                Am = np.zeros((16, 4)); Bm = np.zeros((4, 16)); Am[r, g] = av[:, s]; Bm[g, r] = bv[:, s]
                                a_acc[i] += Am @ Bm
                        db += bv.sum(1)
                for i in range(TMW):
                    m = tg*MPB + wm + WROWS*i
                    for l in range(64):
                        rr, gg = l & 15, l >> 4
                        for q in range(4):
                            row = 16*m + 4*gg + q
                            if row < KK: slab[sp, row*COUT + 16*j + rr] = a_acc[i, gg*4+q, rr]
                if tg == 0 and wm == 0:
                    dbt = np.array([db[rr] + db[rr+16] + db[rr+32] + db[rr+48] for rr in range(16)])
                    slab[sp, KK*COUT + 16*j: KK*COUT + 16*j + 16] = dbt
    tot = slab.sum(0)
    # reference
    Xp = np.zeros((B, H+KS-1, W+KS-1, CIN)); Xp[:, PT:PT+H, PL:PL+W] = X
    ref = np.zeros((KS, KS, CIN, COUT))
    for ky in range(KS):
        for kx in range(KS):
            ref[ky, kx] = np.einsum('bhwc,bhwo->co', Xp[:, ky:ky+ST*(OH-1)+1:ST, kx:kx+ST*(OW-1)+1:ST], dY)
    refv = np.concatenate([ref.reshape(-1), dY.sum((0,1,2))])
    print((CIN, COUT, KS, H, TMW, B, S), 'TG', TG, 'maxerr', np.abs(tot - refv).max(), 'nan', np.isnan(slab).sum(), 'LDS KB', (XSZ + R*WPAD*COS)*4/1024, 'CS', CS, 'COS', COS)
sim(4, 32, 8, 84, 5, 1, 3, ST=4, VALID=True)
sim(32, 64, 4, 20, 4, 2, 3, ST=2, VALID=True)
sim(64, 64, 3, 9, 4, 2, 2, ST=1, VALID=True)
sim(16, 32, 4, 20, 5, 2, 2, ST=2, VALID=True)
sim(32, 32, 5, 42, 5, 1, 2)
