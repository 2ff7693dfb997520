import sys, os, numpy as np, torch
R=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R+'/binius-ntt_amd/python'); sys.path.insert(0, R+'/tests')
import binius_ntt_amd as B, _oracle as O
dev=torch.device('cuda:0')
lh=14
x = O.mt_fill(0xdeadbeef+lh, 1<<lh)
# oracle after stage 13 only
s=O.subspace_evals(lh,0)
def mul(a,b): return O.lib().orc_mul32(int(a),int(b))
y=x.copy().astype(np.uint64)
st=13; half=1<<st
for blk in range((1<<lh)>>(st+1)):
    w=0
    for k in range(lh-1-st):
        if (blk>>k)&1: w^=int(s[st][k])
    for kk in range(half):
        u=blk*(2*half)+kk; v=u+half
        y[u]^=mul(w,y[v]); y[v]^=y[u]
y=y.astype(np.uint32)
os.environ['BN_DEBUG_MAX_PASSES']='1'
ntt=B.AdditiveNTT(B.AdditiveNTTConf(lh,0,B.FanPaarTowerField(5)))
xi=torch.from_numpy(x.view(np.int32)).to(dev); o=torch.zeros_like(xi)
ntt.forward_device(xi,o); torch.cuda.synchronize(); g=o.cpu().numpy().view(np.uint32).copy()
# untranspose each 32-word block
gb=g.reshape(-1,32).copy()
for i in range(gb.shape[0]):
    r=np.ascontiguousarray(gb[i]); O.lib().orc_bitslice_untranspose32(r); gb[i]=r
gc=gb.reshape(-1)
bad=np.nonzero(gc!=y)[0]
print('after pass1 mismatches',len(bad), bad[:8])
print('input==y?', (x==y).sum())
