import sys; sys.path.insert(0,'.')
import torch, numpy as np
from rustfs_amd import Erasure, RSG_RECONSTRUCT_MISSING
from oracle import oracle as O
k,m,S,n=8,4,131072,16
e=Erasure(k,m,k*S)
for miss in [(0,3,5),(0,1,2),(0,3,5,7)]:
  for nn in [1,2,16]:
    g=torch.Generator(device='cuda').manual_seed(3)
    st=torch.zeros((nn,k+m,S),dtype=torch.uint8,device='cuda')
    st[:,:k]=torch.randint(0,256,(nn,k,S),dtype=torch.uint8,device='cuda',generator=g)
    e.encode_batch(st); ref=st.clone()
    for i in miss: st[:,i]=0x5A
    e.reconstruct_batch(st,[i not in miss for i in range(k+m)],RSG_RECONSTRUCT_MISSING)
    torch.cuda.synchronize()
    d=(st!=ref)
    if d.any():
      idx=d.nonzero()
      print(miss, nn, 'bad count',int(d.sum()), 'stripes',sorted(set(idx[:,0].tolist()))[:10],'shards',sorted(set(idx[:,1].tolist())),'bytes min/max',int(idx[:,2].min()),int(idx[:,2].max()))
      h=ref[0].cpu().numpy().copy(); b=st[0].cpu().numpy()
      rows=[h[i].copy() for i in range(k+m)]
    else: print(miss,nn,'ok')
