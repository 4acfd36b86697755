# numpy emulation of dconv_body for DBwdUnpool (dX of a stride-1 SAME conv): flipped-weight staging,
# pads KH-1-PT, pixel-quad units; checked against dX = sum over taps of dY shifted x W^T (no epilogue)
import numpy as np
def sim(G, WM, WN, TMW, CK, B=1):
    CIN, COUT, KS, H = G
    pt_tot = KS - 1; PT = pt_tot // 2
    CI, CO, KH, KW = COUT, CIN, KS, KS
    PTb = KH - 1 - PT; PLb = PTb
    QT = CI // 4; TAPS = KH * KW; KK = TAPS * CI; KP = (KK + 15) // 16 * 16; KC = KP // 16
    TN = CO // 16; TNW = TN // WN; UPB = WM * TMW * 4; NPIX = H * H; U = (NPIX + 3) // 4; BPI = (U + UPB - 1) // UPB
    RSPAN = min((4 * UPB - 1) // H + 2, H); RIN = RSPAN + KH - 1; WP = H + KW - 1; CS = CI + 4 if CI % 16 == 0 else CI
    WPX = WP + (4 if (CI, H, UPB) == (32, 42, 32) else 0)
    CS = 40 if (CI, H, UPB) == (32, 42, 32) else CS
    ASZ = (RIN * WPX * CS + 3) // 4 * 4; CK = CK if CK > 0 else KP; TPC = CK // CI; CKC = CK // 16; NCH = KC // CKC
    rs = np.random.RandomState(1)
    dY = rs.randn(B, H, H, COUT); Wt = rs.randn(KS, KS, CIN, COUT)
    Wf = Wt.reshape(-1)
    def wquad(k, n):
        t, c = divmod(k, CI); tf = (KH - 1 - t // KW) * KW + (KW - 1 - t % KW)
        o = (tf * CIN + n) * COUT + c
        return Wf[o:o + 4]
    out = np.full((B, NPIX, CO), np.nan)
    for bid in range(B * BPI):
        b = bid // BPI; u0 = (bid - b * BPI) * UPB; oy0 = (4 * u0) // H
        As = np.full(ASZ, np.nan)
        for item in range(RIN * WP * QT):
            pix, cq = divmod(item, QT); pr, pc = divmod(pix, WP)
            iy = oy0 - PTb + pr; ix = pc - PLb
            ok = 0 <= iy < H and 0 <= ix < H
            As[(pr * WPX + pc) * CS + 4 * cq:(pr * WPX + pc) * CS + 4 * cq + 4] = dY[b, iy, ix, 4 * cq:4 * cq + 4] if ok else 0
        for w in range(WM * WN):
            wm, wn = w // WN, w % WN
            lanes = np.arange(64); r = lanes & 15; g = lanes >> 4
            acc = np.zeros((TMW, TNW, 16, 16))
            abase = []
            for i in range(TMW):
                u = np.minimum(u0 + (wm * TMW + i) * 4 + (r >> 2), U - 1); q = r & 3
                px = np.minimum(4 * u + q, NPIX - 1); oy = px // H; ox = px - oy * H
                abase.append(((oy - oy0) * WPX + ox) * CS)
            for c in range(NCH):
                Bs = np.full(CKC * TN * 256, np.nan)
                for item in range((CK // 4) * CO):
                    kq, n = divmod(item, CO)
                    v = wquad(c * CK + 4 * kq, n)
                    kcl, gg, j, rr = kq >> 2, kq & 3, n >> 4, n & 15
                    o = ((kcl * TN + j) * 64 + gg * 16 + rr) * 4; Bs[o:o + 4] = v
                for kcl in range(CKC):
                    t = c * TPC + (4 * kcl) // QT
                    ao = ((t // KW) * WPX + t % KW) * CS + 4 * ((4 * kcl) % QT) + 4 * g
                    for i in range(TMW):
                        a = np.stack([As[abase[i] + ao + s] for s in range(4)], 1)
                        for j in range(TNW):
                            bb = np.stack([Bs[((kcl * TN + wn * TNW + j) * 64 + lanes) * 4 + s] for s in range(4)], 1)
                            for s in range(4):
                                Am = np.zeros((16, 4)); Bm = np.zeros((4, 16)); Am[r, g] = a[:, s]; Bm[g, r] = bb[:, s]
                                acc[i, j] += Am @ Bm
            for i in range(TMW):
                for j in range(TNW):
                    for l in range(64):
                        rr, gg = l & 15, l >> 4
                        u = u0 + (wm * TMW + i) * 4 + gg
                        if u >= U: continue
                        n = (wn * TNW + j) * 16 + rr
                        for q in range(4):
                            p = 4 * u + q
                            if p < NPIX: out[b, p, n] = acc[i, j, gg * 4 + q, rr]
    # reference dX: forward y[oy,ox,co] = sum x[oy-PT+ky, ox-PT+kx, ci] W[ky,kx,ci,co]
    ref = np.zeros((B, H, H, CIN))
    for ky in range(KS):
        for kx in range(KS):
            for oy in range(H):
                for ox in range(H):
                    iy, ix = oy - PT + ky, ox - PT + kx
                    if 0 <= iy < H and 0 <= ix < H:
                        ref[:, iy, ix] += dY[:, oy, ox] @ Wt[ky, kx].T
    ref = ref.reshape(B, NPIX, CIN)
    print(G, (WM, WN, TMW, CK), 'maxerr', np.nanmax(np.abs(out - ref)), 'nan', np.isnan(out).sum(), 'LDS KB', (ASZ + (2 if NCH > 1 else 1) * CKC * TN * 256) * 4 / 1024)
sim((32, 32, 5, 42), 4, 2, 2, 32)
