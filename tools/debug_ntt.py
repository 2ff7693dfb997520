import sys, os, numpy as np, torch
R=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R+'/binius-ntt_amd/python'); sys.path.insert(0, R+'/tests')
import binius_ntt_amd as B, _oracle as O
dev=torch.device('cuda:0')
for fb,lh,r in [(32,14,0),(128,14,0),(32,13,1),(32,15,0)]:
    lim=fb//32
    x = O.mt_fill(0xdeadbeef+lh, (1<<lh)*lim)
    ntt=B.AdditiveNTT(B.AdditiveNTTConf(lh,r,B.FanPaarTowerField(5 if fb==32 else 7)))
    xi=torch.from_numpy(x.view(np.int32)).to(dev); y=torch.empty(x.size<<r,dtype=torch.int32,device=dev)
    ntt.forward_device(xi,y); torch.cuda.synchronize(); g=y.cpu().numpy().view(np.uint32)
    e = O.antt32(x,lh,r) if fb==32 else O.antt128(x.reshape(-1,4),lh,r).reshape(-1)
    bad=np.nonzero(g!=e)[0]
    print(fb,lh,r,'variant',ntt.variant(),'mismatch',len(bad),'of',g.size, bad[:10])
    if len(bad):
        # is output equal to oracle with only low 13 stages / only stage 13?
        print(' first bad idx bits', [bin(b) for b in bad[:4]])
