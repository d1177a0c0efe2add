"""Diagnose the fp16-pair fp32 kernel (news_x2.hip): x2 and the fp32-MFMA kernel against float64.

    python tools/x2_diag.py [B] [L] [d] [C] [K]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import news, synthetic  # noqa: E402

dev = "cuda:0"
B, L, d, C, K = (int(x) for x in (sys.argv[1:6] + ["300", "50", "768", "40", "32"][len(sys.argv) - 1:]))
n_news, Dc = 5000, 200
g = torch.Generator().manual_seed(5)
table = (torch.randn((n_news, d), generator=g) / d ** 0.5).to(dev)
lens = torch.randint(0, L + 1, (B,), generator=g)
mask = (torch.arange(L)[None, :] >= (L - lens)[:, None])
hid = torch.randint(1, n_news, (B, L), generator=g)
hid[~mask] = 0
cid = torch.randint(1, n_news, (B, C), generator=g)
hid, mask, cid = hid.to(dev), mask.to(dev), cid.to(dev)
W1, Q, W2 = synthetic.init_weights(5, d, Dc, K, device=dev)
T = table.double().cpu()
E, Cd = T[hid.cpu().long()], T[cid.cpu().long()]
w1, q, w2 = (x.double().cpu() for x in (W1, Q, W2))
s = torch.tanh(E @ w1.T) @ q.T
s = s.masked_fill(~mask.cpu()[:, :, None], 1e-30)
A = torch.softmax(s, dim=1)                       # [B, L, K]
mui = torch.einsum("blk,bld->bkd", A, E)
x = torch.nn.functional.gelu(mui @ w2.T)
m = Cd @ mui.transpose(1, 2)
ref_w = (torch.softmax(Cd @ x.transpose(1, 2), dim=-1) * m).sum(-1)
ref_max = m.max(-1).values
for kern in ("mfma32", "x2"):
    os.environ["MINER_NEWS_FP32"] = kern
    nt = news.precompute(table, W1, Q, W2)
    for st, ref in (("weighted", ref_w), ("max", ref_max)):
        sc, mu = news.score(nt, hid, mask, cid, score_type=st, return_user=True)
        torch.cuda.synchronize()
        e = (sc.double().cpu() - ref).abs() / ref.pow(2).mean().sqrt()
        em = (mu.double().cpu() - mui).abs() / mui.pow(2).mean().sqrt()
        b, k, c = [int(v) for v in torch.nonzero(em == em.max())[0]]
        print(f"{kern} {st}: scores max {float(e.max()):.2e} rms {float(e.pow(2).mean().sqrt()):.2e} x rms(ref); "
              f"mui max {float(em.max()):.2e} at b={b} k={k} col={c} (A max {float(A[b, :, k].max()):.3f}, "
              f"len {int(mask[b].sum())}, |mui| {float(mui[b, k, c].abs()):.3e}, rms {float(mui.pow(2).mean().sqrt()):.3e}); "
              f"mui elems > 1e-5: {int((em > 1e-5).sum())}", flush=True)

# error pattern of the last (x2) mui
em = (mu.double().cpu() - mui).abs() / mui.pow(2).mean().sqrt()
bad = em > 1e-5
print("bad elems per k:", bad.sum((0, 2)).tolist())
print("bad elems per col % 64:", bad.sum((0, 1)).view(-1, 64).sum(0).tolist())
print("bad elems per chunk:", bad.sum((0, 1)).view(-1, 64).sum(1).tolist())
lens_c = mask.sum(1).cpu()
bi = bad.sum((1, 2))
print("impressions with bad elems:", int((bi > 0).sum()), "lens of those:", sorted(lens_c[bi > 0].tolist())[:40])
print("lens of clean:", sorted(lens_c[bi == 0].tolist())[:60])
# representation check: hi/lo split of E and A in f64
sE = float(nt.x2.table_unit[0])
Es = T * sE
Eh = Es.float().half().double()
El = (Es - Eh).float().half().double()
As = (A * 16384.0)
Ah = As.float().half().double()
Al = (As - Ah).float().half().double()
Erep = T[hid.cpu().long()] * 0 + (Eh + El)[hid.cpu().long()]
mrep = (torch.einsum("blk,bld->bkd", Ah, Erep) + torch.einsum("blk,bld->bkd", Al, Eh[hid.cpu().long()])) / (sE * 16384.0)
er = (mrep - mui).abs() / mui.pow(2).mean().sqrt()
print(f"representation-only mui error max {float(er.max()):.2e}")
print("bad (b, k):", [(int(b), int(k)) for b, k in torch.nonzero(bad.any(2))])
outs = []
for rep in range(4):
    sc, mu2 = news.score(nt, hid, mask, cid, return_user=True)
    torch.cuda.synchronize()
    outs.append(mu2.double().cpu())
    em2 = (outs[-1] - mui).abs() / mui.pow(2).mean().sqrt()
    print(f"rep {rep}: bad (b, k):", [(int(b), int(k)) for b, k in torch.nonzero((em2 > 1e-5).any(2))])
print("reps bit-identical:", all(torch.equal(outs[0], o) for o in outs[1:]))
Eb_all = T[hid.cpu().long()]
for b, k in [(94, 7), (148, 20), (173, 29), (198, 3)]:
    delta = outs[0][b, k] - mui[b, k]
    Eb = Eb_all[b]                                    # [L, d]
    sol = torch.linalg.lstsq(Eb.T, delta.unsqueeze(1)).solution.squeeze(1)   # dA per slot
    top = torch.argsort(sol.abs(), descending=True)[:4]
    print(f"(b={b}, k={k}) len {int(mask[b].sum())}: dA top slots {[(int(t), float(sol[t]), float(A[b, t, k])) for t in top]} "
          f"resid {float((Eb.T @ sol - delta).norm() / delta.norm()):.2e}; logits of k: max {float(s[b, :, k].max()):.3f} "
          f"min {float(s[b, :, k].min()):.3f}")
P_all = nt.proj.double().cpu()
for b, k in [(94, 7), (148, 20)]:
    delta = outs[0][b, k] - mui[b, k]
    print(f"(b={b},k={k}) |delta|/|mui| {float(delta.norm() / mui[b, k].norm()):.2e}; delta first 8: {[float(x) for x in delta[:8]]}")
    basis = {"E": Eb_all[b], "proj": P_all[hid.cpu().long()[b]], "cand": T[cid.cpu().long()[b]],
             "mui_all_k": mui[b], "table": T}
    for nm, Bm in basis.items():
        sol = torch.linalg.lstsq(Bm.T, delta.unsqueeze(1)).solution.squeeze(1)
        print(f"   basis {nm} ({Bm.shape[0]} rows): resid {float((Bm.T @ sol - delta).norm() / delta.norm()):.3e}")
    cos = (T @ delta) / (T.norm(dim=1) * delta.norm())
    j = int(cos.abs().argmax())
    print(f"   best single table row {j} cos {float(cos[j]):.4f}; is it in the history? {j in hid.cpu()[b].tolist()}, cand? {j in cid.cpu()[b].tolist()}")
