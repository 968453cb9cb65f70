import os, sys, time
sys.path.insert(0, "/root/repo")
import numpy as np, torch
from wavernn_amd import synthetic as syn
from wavernn_amd.loop import FatchordLoop
d = syn.DEFAULT_MOL
state = syn.make_fatchord_state(d, 0)
mels, aux = syn.make_conditioning(1, 5000, d.feat_dims, d.res_out_dims, 5)
cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).cuda()
loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
loop.set_weights(state)
for reps in (8, 2, 4, 8, 16, 32):
    os.environ["WRNN_REPLICAS"] = str(reps)
    ts = []
    for _ in range(3):
        loop.generate(cond, seed=1); ts.append(loop.elapsed_ms() * 1e3 / 5000)
    print(f"replicas {reps:3d}: {min(ts):.2f} us/step (runs {', '.join(f'{x:.2f}' for x in ts)})", flush=True)
