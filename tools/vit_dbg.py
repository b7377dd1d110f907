import sys, time, torch
sys.path.insert(0, '/root/repo')
import deepfake_amd
from deepfake_amd.vit_gcn import DeepfakeModel
from deepfake_amd.detector import chain_adjacency
from deepfake_amd.weights import deterministic_init_
dev = torch.device('cuda', 0)
for B in [1, 4, 16]:
    N = 8
    m = DeepfakeModel(compute_dtype='bf16'); deterministic_init_(m, seed=0); m = m.to(dev).train()
    x = torch.rand(B, N, 3, 224, 224, device=dev)
    a = torch.from_numpy(chain_adjacency(N)).float().to(dev).expand(B, N, N).contiguous()
    t0 = time.time()
    out = m(x, a); torch.cuda.synchronize(); t1 = time.time()
    out.sum().backward(); torch.cuda.synchronize(); t2 = time.time()
    print(B, 'fwd', round(t1 - t0, 3), 'bwd', round(t2 - t1, 3), flush=True)
