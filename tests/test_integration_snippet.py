"""INTEGRATION.md section B — the ctypes binding a reference maintainer would add to
models/fatchord_version.py — executed as written (only the library path is made absolute), on a
module with the reference constructor and state_dict keys (the drop-in WaveRNN; not the
reference itself).  Without a GPU the loop call must fail through wrnn_create's status; on the
MI355X it runs the persistent kernel and matches the C oracle (injected noise) and the package's
own FatchordLoop (Philox)."""
import ctypes
import os
import re

import numpy as np

import pytest
import torch

from wavernn_amd import _native as nat
from wavernn_amd import synthetic as syn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _snippet_ns():
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = text[text.index("## B."):text.index("## C.")]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    code = code.replace('"wavernn_amd/_lib/libwavernn_amd.so"', repr(nat.LIB_PATH))
    ns = {}
    exec(compile(code, "INTEGRATION.md#B", "exec"), ns)
    return ns


def _model(d):
    from wavernn_amd.fatchord_version import WaveRNN
    return WaveRNN(**d.ctor_kwargs())


@pytest.mark.parametrize("d", [syn.DEFAULT_MOL, syn.DEFAULT_RAW, syn.TINY_MOL])
def test_snippet_config_fields(d):
    ns = _snippet_ns()
    cfg = ns["_wrnn_cfg"](_model(d))
    assert ns["WRNN_ABI_VERSION"] == nat.ABI_VERSION
    hdr = open(os.path.join(REPO, "include", "wavernn_amd.h")).read()
    assert f"#define WRNN_ABI_VERSION {nat.ABI_VERSION}" in hdr
    assert [f for f, _ in ns["_Cfg"]._fields_] == [f for f, _ in nat.Config._fields_]
    want = dict(abi_version=nat.ABI_VERSION, mode=nat.MODE_MOL if d.mode == "MOL" else nat.MODE_RAW,
                rnn_dims=d.rnn_dims, fc_dims=d.fc_dims, aux_dims=d.aux_dims, feat_dims=d.feat_dims,
                n_classes=d.n_classes, grid=0, timeout_ms=0)
    assert {f: getattr(cfg, f) for f in want} == want


def test_snippet_tensor_array():
    ns = _snippet_ns()
    d = syn.DEFAULT_MOL
    m = _model(d)
    ts, keep = ns["_wrnn_tensors"](m)
    sd = m.state_dict()
    assert [t.name.decode() for t in ts] == ns["LOOP_KEYS"] == list(__import__("wavernn_amd.loop").loop.LOOP_KEYS)
    for t, k, kept in zip(ts, ns["LOOP_KEYS"], keep):
        assert t.numel == sd[k].numel() and t.on_device == 0 and t.data == kept.data_ptr()


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_snippet_fails_cleanly_without_gpu():
    ns = _snippet_ns()
    m = _model(syn.DEFAULT_MOL)
    mels, aux = torch.zeros(1, 10, 80), torch.zeros(1, 10, 128)
    with pytest.raises(AssertionError) as e:
        ns["_hip_loop"](m, mels, aux, seed=1)
    assert e.value.args and e.value.args[0]     # wrnn_last_error's message
    # the handle path itself: create fails with a status, the (possibly null) handle is released
    lib = ns["_lib"]
    h = ctypes.c_void_p()
    rc = lib.wrnn_create(ctypes.byref(ns["_wrnn_cfg"](m)), 0, ctypes.byref(h))
    assert rc < 0
    lib.wrnn_destroy(h)


@pytest.mark.gpu
@pytest.mark.parametrize("d", [syn.DEFAULT_MOL, syn.TINY_MOL])
def test_snippet_hip_loop_on_gpu(d):
    from oracle import oracle
    from tests.golden import fixtures as gf
    from wavernn_amd.loop import FatchordLoop
    ns = _snippet_ns()
    m = _model(d)
    state = syn.make_fatchord_state(d, 21)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    m = m.to("cuda")
    B, L = 2, 700
    mels, aux = syn.make_conditioning(B, L, d.feat_dims, d.res_out_dims, 22)
    noise = syn.make_noise(d.mode, B, L, d.n_classes, 23)
    gm, ga = torch.from_numpy(mels).cuda(), torch.from_numpy(aux).cuda()
    out = ns["_hip_loop"](m, gm, ga, seed=1, noise=torch.from_numpy(noise).cuda())
    ref, _ = oracle.fatchord_loop(state, d.mode, mels, aux, noise)
    assert np.abs(out.cpu().numpy() - ref).max() <= gf.MOL_TOL
    # Philox: the snippet and the package's binding run the same launch
    out_p = ns["_hip_loop"](m, gm, ga, seed=99)
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    loop.set_weights(state)
    cond = torch.cat([gm, ga], 2).transpose(0, 1).contiguous()
    y, _ = loop.generate(cond, seed=99)
    assert torch.equal(out_p, y)
    loop.close()
