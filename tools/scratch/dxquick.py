import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from wavernn_amd import _native
if os.environ.get("TIME_DM_LIB"): _native.LIB_PATH = os.environ["TIME_DM_LIB"]
from oracle import oracle
from wavernn_amd import synthetic as syn
from wavernn_amd.loop import DeepmindLoop
d = syn.DEFAULT_DM
for B, L in ((1, 60), (4, 60)):
    st = syn.make_deepmind_state(d, 11)
    nz = syn.make_dm_noise(B, L, d.quantisation, 12)
    c, f, ref = oracle.deepmind_loop(st, B, L, nz)
    lp = DeepmindLoop(d.hidden_size, d.quantisation); lp.set_weights(st)
    _, comb = lp.generate(B, L, noise=torch.from_numpy(nz).cuda())
    got = comb.cpu().numpy().astype(np.int64)
    gc, gf = (got + 32768) // 256, (got + 32768) % 256
    for b in range(B):
        bad = np.nonzero(got[b] != ref[b])[0]
        print(os.path.basename(_native.LIB_PATH), "B", B, "row", b, "first bad", bad[:3], "coarse ok", (gc[b][:bad[0]+1] == c[b][:bad[0]+1]).tolist()[-2:] if len(bad) else "-", "fine", (gf[b][:bad[0]+1]==f[b][:bad[0]+1]).tolist()[-2:] if len(bad) else "-")
    lp.close()
