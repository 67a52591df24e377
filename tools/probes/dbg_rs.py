import sys, numpy as np, torch
sys.path.insert(0, '.')
from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine
from tests.oracle_lib import Oracle
o = Oracle()
bs, t = 512, 3
n, k, _ = o.rs_sizes(bs, t)
eng = EccEngine(ECC_REED_SOLOMON, bs, t)
nb = 249 * 2
data = np.zeros((nb, k), np.uint8)
for j in range(249):
    data[j, j] = 1
    data[249 + j, j] = 0x80
data = data.reshape(-1)
raw = torch.zeros(nb * n, dtype=torch.uint8, device='cuda')
eng.encode(torch.from_numpy(data).cuda(), raw, nblocks=nb)
torch.cuda.synchronize()
got = raw.cpu().numpy().reshape(nb, n); ref = o.rs_encode(bs, t, data).reshape(nb, n)
badj = [j for j in range(nb) if not np.array_equal(got[j], ref[j])]
print('bad impulses', len(badj), badj[:60])
for j in badj[:4]:
    print(j, 'got', got[j, :6], 'ref', ref[j, :6])
