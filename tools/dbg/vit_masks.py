"""Debug: dump the Viterbi ballot masks of one small case and compare with numpy."""
import sys, os
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "vq-vae-hmm-model_amd")); sys.path.insert(0, ROOT)
import vqhmm
from vqhmm import _ext
from oracle import c_oracle

K, B, T = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rng = np.random.default_rng(0)
def lsm(a): m = a.max(-1, keepdims=True); return a - m - np.log(np.exp(a - m).sum(-1, keepdims=True))
log_pi = lsm(rng.standard_normal(K)).astype(np.float32)
log_A = lsm(rng.standard_normal((B, T, K, K)) * 1.5).astype(np.float32)
em = lsm(rng.standard_normal((B, T, K)) * 2).astype(np.float32)
L = np.full(B, T, np.int64)
lib = _ext.load()
g = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
tp, tA, te, tL = g(log_pi), g(log_A), g(em), g(L)
path = torch.empty(B, T, dtype=torch.int32, device="cuda"); score = torch.empty(B, device="cuda")
nb = lib.vqhmm_viterbi_workspace_size(B, T, K)
ws = torch.zeros(nb, dtype=torch.uint8, device="cuda")
rc = lib.vqhmm_viterbi_f32(_ext.ptr(tp), _ext.ptr(tA), _ext.ptr(te), _ext.ptr(tL), B, T, K, _ext.ptr(path), _ext.ptr(score), _ext.ptr(ws), nb, _ext.stream_ptr())
torch.cuda.synchronize()
print("rc", rc)
masks = ws.cpu().numpy().view(np.uint64)
rp, rs = c_oracle.viterbi(log_pi, log_A, em, L)
print("gpu path[0][:20]", path.cpu().numpy()[0][:20])
print("ref path[0][:20]", rp[0][:20])
print("score", score.cpu().numpy()[:4], rs[:4])
KP = 2 if K <= 2 else 4 if K <= 4 else 8
G = KP * KP
# expected masks for seq 0 (wave 0): delta recursion
d = log_pi + em[0, 0]
for t in range(1, min(T, 8)):
    v = d[:, None] + log_A[0, t]  # (i, j)
    m = v.max(0)
    eq = v == m[None, :]
    bits = 0
    for gg in range(G):
        i, j = (gg // KP, gg % KP) if t % 2 == 0 else (gg % KP, gg // KP)
        if i < K and j < K and eq[i, j]:
            bits |= 1 << gg
    print(t, "gpu mask %016x" % int(masks[t]), "expect(seq0 bits) %x" % bits)
    d = m + em[0, t]
