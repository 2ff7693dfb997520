import sys, os, numpy as np, torch
R=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R+'/binius-ntt_amd/python'); sys.path.insert(0, R+'/tests')
import binius_ntt_amd as B, _oracle as O
dev=torch.device('cuda:0')
lh=int(sys.argv[1]) if len(sys.argv)>1 else 14
x = O.mt_fill(0xdeadbeef+lh, 1<<lh)
s=O.subspace_evals(lh,0)
M=O.lib().orc_mul32
y=x.astype(np.uint64).copy()
ntt=B.AdditiveNTT(B.AdditiveNTTConf(lh,0,B.FanPaarTowerField(5)))
xi=torch.from_numpy(x.view(np.int32)).to(dev)
for st in range(lh-1,-1,-1):
    half=1<<st
    for blk in range((1<<lh)>>(st+1)):
        w=0
        for k in range(lh-1-st):
            if (blk>>k)&1: w^=int(s[st][k])
        base=blk*2*half
        for kk in range(half):
            u=base+kk; v=u+half
            y[u]^=M(w,int(y[v])); y[v]^=y[u]
    if st>=13: continue
    os.environ['BN_DEBUG_STOP_STAGE']=str(st)
    o=torch.zeros_like(xi); ntt.forward_device(xi,o); torch.cuda.synchronize(); g=o.cpu().numpy().view(np.uint32)
    bad=np.nonzero(g!=y.astype(np.uint32))[0]
    print('after stage',st,'mismatches',len(bad),bad[:6]); sys.stdout.flush()
    if len(bad): break
