# numpy emulation of dconv_body for DFwd of a strided VALID conv (non-pooled quads), vs a direct conv
import numpy as np
def run(CIN, COUT, KS, S, H, WM, WN, TMW, CK, B=2):
    W=H; OH=(H-KS)//S+1; OW=OH; PT=PL=0
    QT=CIN//4; TAPS=KS*KS; KK=TAPS*CIN; KP=(KK+15)//16*16; KC=KP//16
    TN=COUT//16; TNW=TN//WN; UPB=WM*TMW*4; NPIX=OH*OW; U=(NPIX+3)//4; BPI=(U+UPB-1)//UPB
    RSPAN=min((4*UPB-1)//OW+2, OH); RIN=(RSPAN-1)*S+KS; WP=(OW-1)*S+KS; WPX=WP
    CS=CIN+4 if CIN%16==0 else CIN; ASZ=(RIN*WPX*CS+3)//4*4
    CK=CK if CK>0 else KP; TAPAL=QT%4==0 and CK%CIN==0; TPC=CK//CIN if TAPAL else 0; CKC=CK//16; NCH=KC//CKC
    rs=np.random.RandomState(3); X=rs.rand(B,H,W,CIN); Wt=rs.randn(KS,KS,CIN,COUT)*0.1; bias=rs.randn(COUT)*0.1
    Wf=Wt.reshape(-1,COUT); Y=np.full((B,NPIX,COUT),np.nan)
    for bid in range(B*BPI):
        b=bid//BPI; u0=(bid-b*BPI)*UPB; oy0=(4*u0)//OW
        As=np.full(ASZ,np.nan)
        for item in range(RIN*WP*QT):
            pix,cq=divmod(item,QT); pr,pc=divmod(pix,WP)
            iy=oy0*S-PT+pr; ix=pc-PL; ok=0<=iy<H and 0<=ix<W
            As[(pr*WPX+pc)*CS+4*cq:(pr*WPX+pc)*CS+4*cq+4]=X[b,iy,ix,4*cq:4*cq+4] if ok else 0
        for w in range(WM*WN):
            wm,wn=w//WN,w%WN; lanes=np.arange(64); r=lanes&15; g=lanes>>4
            acc=np.zeros((TMW,TNW,16,16)); abase=[]
            for i in range(TMW):
                u=np.minimum(u0+(wm*TMW+i)*4+(r>>2),U-1); q=r&3
                px=np.minimum(4*u+q,NPIX-1); oy=px//OW; ox=px-oy*OW
                abase.append(((oy-oy0)*S*WPX+ox*S)*CS)
            for c in range(NCH):
                Bs=np.full(CKC*TN*256,np.nan)
                for item in range((CK//4)*COUT):
                    kq,n=divmod(item,COUT); k=c*CK+4*kq
                    v=[Wf[min(k+s,KK-1),n] if k+s<KK else 0 for s in range(4)]
                    kcl,gg,j,rr=kq>>2,kq&3,n>>4,n&15; o=((kcl*TN+j)*64+gg*16+rr)*4; Bs[o:o+4]=v
                for kcl in range(CKC):
                    kc=c*CKC+kcl
                    if TAPAL:
                        t=c*TPC+(4*kcl)//QT; ao=((t//KS)*WPX+t%KS)*CS+4*((4*kcl)%QT)+4*g
                    else:
                        q4=4*kc+g; t0=q4//QT; cq=q4-t0*QT; t=np.minimum(t0,TAPS-1); ky=t//KS; kx=t-ky*KS; ao=(ky*WPX+kx)*CS+4*cq
                    for i in range(TMW):
                        a=np.stack([As[abase[i]+ao+s] for s in range(4)],1)
                        for j in range(TNW):
                            bb=np.stack([Bs[((kcl*TN+wn*TNW+j)*64+lanes)*4+s] for s in range(4)],1)
                            for s in range(4):
                                Am=np.zeros((16,4)); Bm=np.zeros((4,16)); Am[r,g]=a[:,s]; Bm[g,r]=bb[:,s]; acc[i,j]+=Am@Bm
            for i in range(TMW):
                for j in range(TNW):
                    for l in range(64):
                        rr,gg=l&15,l>>4; u=u0+(wm*TMW+i)*4+gg
                        if u>=U: continue
                        n=(wn*TNW+j)*16+rr
                        for q in range(4):
                            p=4*u+q
                            if p<NPIX: Y[b,p,n]=max(acc[i,j,gg*4+q,rr]+bias[n],0)
    ref=np.zeros((B,OH,OW,COUT))
    for ky in range(KS):
        for kx in range(KS):
            ref+=np.einsum('bhwc,co->bhwo', X[:,ky:ky+S*(OH-1)+1:S, kx:kx+S*(OW-1)+1:S], Wt[ky,kx])
    ref=np.maximum(ref+bias,0).reshape(B,NPIX,COUT)
    print((CIN,COUT,KS,S,H),(WM,WN,TMW,CK),'maxerr',np.nanmax(np.abs(Y-ref)),'nan',np.isnan(Y).sum(),'LDS KB',(ASZ+(2 if NCH>1 else 1)*CKC*TN*256)*4/1024)
run(4,32,8,4,84,4,1,1,0)
run(32,64,4,2,20,2,4,1,32)
run(64,64,3,1,9,2,4,1,64)
