"""Checkpoint writer / restorer (`utils/checkpoints.py:29-132`, `utils/paths.py:5-71`) on CPU:
directory layout and file names, latest + named pairs, the broken-pair rule, create_if_missing
with init weights, and an Adam state round trip through the safe loader."""
import numpy as np
import pytest
import torch

from wavernn_amd import synthetic as syn
from wavernn_amd.checkpoints import Paths, get_checkpoint_paths, restore_checkpoint, save_checkpoint
from wavernn_amd.fatchord_version import WaveRNN


def _trained(seed):
    d = syn.TINY_RAW
    m = WaveRNN(**d.ctor_kwargs())
    state = syn.make_fatchord_state(d, seed)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(seed)
    for p in m.parameters():
        p.grad = torch.randn(p.shape, generator=g)
    opt.step()
    m.step += 7
    return m, opt


def _fresh():
    m = WaveRNN(**syn.TINY_RAW.ctor_kwargs())
    return m, torch.optim.Adam(m.parameters(), lr=1e-3)


def _same_model(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    return sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sa)


def test_paths_layout(tmp_path):
    p = Paths(tmp_path / 'data', 'ljspeech_mol', 'ljspeech_lsa', base=tmp_path)
    assert p.voc_latest_weights == tmp_path / 'checkpoints' / 'ljspeech_mol.wavernn' / 'latest_weights.pyt'
    assert p.tts_latest_optim == tmp_path / 'checkpoints' / 'ljspeech_lsa.tacotron' / 'latest_optim.pyt'
    assert p.get_voc_named_weights('x') == p.voc_checkpoints / 'x_weights.pyt'
    for d in (p.quant, p.mel, p.gta, p.voc_checkpoints, p.voc_output, p.tts_attention, p.tts_mel_plot):
        assert d.is_dir()
    q = Paths(tmp_path / 'd2', 'v', 't', base=tmp_path / 'b2', ignore_tts=True)
    assert q.voc_checkpoints.is_dir() and not q.tts_checkpoints.exists()
    assert get_checkpoint_paths('voc', p) == (p.voc_latest_weights, p.voc_latest_optim, p.voc_checkpoints)
    with pytest.raises(NotImplementedError):
        get_checkpoint_paths('gan', p)


def test_save_restore_latest_and_named(tmp_path):
    p = Paths(tmp_path / 'data', 'v', 't', base=tmp_path)
    m, opt = _trained(1)
    save_checkpoint('voc', p, m, opt, name='wave_step7K', is_silent=True)
    assert p.voc_latest_weights.exists() and p.voc_latest_optim.exists()
    assert p.get_voc_named_weights('wave_step7K').exists() and p.get_voc_named_optim('wave_step7K').exists()

    for name in (None, 'wave_step7K'):
        m2, opt2 = _fresh()
        restore_checkpoint('voc', p, m2, opt2, name=name)
        assert _same_model(m, m2) and m2.get_step() == m.get_step()
        s1, s2 = opt.state_dict(), opt2.state_dict()
        assert s1['param_groups'] == s2['param_groups']
        for k in s1['state']:
            for f in ('exp_avg', 'exp_avg_sq', 'step'):
                assert torch.equal(s1['state'][k][f], s2['state'][k][f])


def test_broken_pair_and_missing(tmp_path):
    p = Paths(tmp_path / 'data', 'v', 't', base=tmp_path)
    m, opt = _fresh()
    with pytest.raises(FileNotFoundError):
        restore_checkpoint('voc', p, m, opt)
    save_checkpoint('voc', p, m, opt, is_silent=True)
    p.voc_latest_optim.unlink()
    with pytest.raises(FileNotFoundError):
        save_checkpoint('voc', p, m, opt, is_silent=True)
    with pytest.raises(FileNotFoundError):
        restore_checkpoint('voc', p, m, opt, name='nope')


def test_create_if_missing_with_init_weights(tmp_path):
    p = Paths(tmp_path / 'data', 'v', 't', base=tmp_path)
    src, _ = _trained(3)
    init = tmp_path / 'init.pyt'
    src.save(init)
    m, opt = _fresh()
    restore_checkpoint('voc', p, m, opt, create_if_missing=True, init_weights_path=init)
    assert m.get_step() == 0
    sd_m, sd_s = m.state_dict(), src.state_dict()
    assert all(torch.equal(sd_m[k], sd_s[k]) for k in sd_m if k != 'step')
    assert p.voc_latest_weights.exists() and p.voc_latest_optim.exists()
