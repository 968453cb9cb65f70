"""Headline benchmark: WaveRNN MoL (rnn_dims 512) generation on MI355X.

Workload (BASELINE.json configs[1]): one 5 s utterance per GPU (synthetic 80-band mel,
T = 401 frames → 110 275 loop steps, 110 000 output samples), unbatched (batch = 1), MoL
sampling, random weights of the 800k-step MoL architecture (hparams.py).  A "step" of this
benchmark is one full `WaveRNN.generate()` of that utterance (upsample → persistent HIP
loop → float64 post-processing).  N GPUs = N ranks, one utterance each (weak scaling; the
utterances are independent, there is no collective in the data path; the finished audio is
gathered to rank 0 over RCCL).

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts its N rank
processes itself (before the parent touches a GPU); under torchrun it is one of them.

Prints ONE JSON line on rank 0.  `roofline` is computed for the persistent loop kernel from
HIP events around its launch; `roofline.traffic` from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE) of this same script run as child processes before the measured run (N = 1; the
committed profile is the labelled fallback); `cpu_baseline` times the reference's own op
sequence as a PyTorch-CPU eager restatement (oracle/torch_cpu.py) on this host's cores over a
bounded slice of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from wavernn_amd import synthetic as syn  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA peak (dense)
MOL_MACS_PER_ROW_STEP = 3825152   # loop MACs per row-step, MoL rnn 512
# an explicitly named committed PMC summary replaces the live passes (labelled in traffic_from); by
# default there is no fallback: when the live passes fail, roofline.traffic is null
PMC_PROFILE = os.environ.get("WRNN_PMC_PROFILE")
SPARSE896_BYTES_PER_STEP = 5536598   # config 4 sparse values + int16 block indices, fp32
DM_BYTES_PER_STEP = 12200196         # config 5 deepmind weights, fp32
DM_MACS_PER_ROW_STEP = 3045952
COND_BYTES_PER_ROW_STEP = 836  # 208 fp32 conditioning + 1 fp32 output
KERNELS = {7: "fatchord_xcdm_kernel (many rows per XCD, MFMA)", 5: "fatchord_xcd_kernel (one XCD, 32 CUs)",
           4: "fatchord_split_kernel", 2: "fatchord_rows_kernel", 1: "fatchord_loop_kernel"}


def loop_weight_bytes(d: syn.FatchordDims) -> int:
    """fp32 bytes of every weight one loop step reads (I, rnn1, rnn2, fc1-3)."""
    r, f, a, nc = d.rnn_dims, d.fc_dims, d.aux_dims, d.n_classes
    n = (r * (d.feat_dims + a + 1) + r) + (3 * r * r * 2 + 6 * r) + (3 * r * (r + a) + 3 * r * r + 6 * r) \
        + (f * (r + a) + f) + (f * (f + a) + f) + (nc * f + nc)
    return 4 * n


def hbm_roofline(bytes_per_step: float, us_per_step: float, note: str) -> dict:
    achieved = bytes_per_step / (us_per_step * 1e-6) / 1e9
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "note": note}


# ------------------------------------------------------------------------ rank launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """One process per GPU, started from this (GPU-untouched) parent: RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* as torchrun sets them, 127.0.0.1 rendezvous.  Returns the first
    non-zero exit code (the other ranks are then stopped), else 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------------- HBM traffic (PMC)
def _under_profiler() -> bool:
    return any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", "")


def pmc_live(timeout_s: float = 240.0):
    """FETCH_SIZE and WRITE_SIZE passes (one counter each, MI355X_MICROARCH.md's recipe) over
    `bench.py --pmc-child` (the headline and configs 2×8 / 3 / 4 / 5 generated once each), run
    as child processes before this process touches the GPU.  Returns the summary record
    (tools/pmc_summary.py) or None when rocprofv3 is absent or a pass fails."""
    exe = shutil.which("rocprofv3")
    if exe is None or _under_profiler():
        return None
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import pmc_summary
    tmp = tempfile.mkdtemp(prefix="wrnn_pmc_")
    try:
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            cmd = [exe, "--pmc", c, "-d", os.path.join(tmp, "pmc_" + c), "-o", "pmc", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-child"]
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True,
                                 env=dict(os.environ, WRNN_BENCH_PMC_CHILD="1"))
            try:
                if p.wait(timeout=timeout_s) != 0:
                    return None
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return None
        return pmc_summary.summarise(tmp)
    except Exception:          # an unreadable summary falls back to the committed profile
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def committed_pmc(path):
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def resolve_traffic(live, profile_path):
    """(traffic record, traffic_from) for the roofline: this run's live PMC passes; else the
    summary named by WRNN_PMC_PROFILE (labelled as such); else (None, reason) — never an older
    kernel's traffic presented as this one's."""
    if live is not None:
        return live, "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this run"
    prof = committed_pmc(profile_path)
    if prof is not None:
        return prof, os.path.relpath(profile_path, REPO) + " (named by WRNN_PMC_PROFILE; live passes unavailable)"
    return None, "unavailable: the live rocprofv3 passes did not run or failed (traffic null)"


# ------------------------------------------------------------------------ other configs
def _mol_model(d, dev, state):
    from wavernn_amd.fatchord_version import WaveRNN
    model = WaveRNN(**d.ctor_kwargs()).to(dev)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    return model


def _timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return out, time.perf_counter() - t


def other_configs(dev, warm: bool = True, cpu_steps: int = 0, threads: int = 1) -> dict:
    """BASELINE configs 1 and 3 on this rank's GPU, through the drop-in API (upsample and
    post-processing included), synthetic inputs, random weights of each architecture:
      1: RAW 9-bit generate(), 1 s unbatched and 5 s fold-batched;
      3: MoL fold-batched generate() of one 60 s utterance (115 folds x 12 100 steps);
    plus the headline architecture serving 8 utterances at once (generate_many, one per XCD) and
    32 at once (the many-row kernel, 4 per XCD: aggregate serving throughput).
    Configs 4 and 5 are utterance batches sharded over the ranks: `sharded_configs`.
    `warm` = an untimed first call per config (the PMC child runs each config once)."""
    res = {}
    sr = 22050
    # config 2 architecture, 8 concurrent unbatched utterances (per-stream latency unchanged)
    d = syn.DEFAULT_MOL
    model = _mol_model(d, dev, syn.make_fatchord_state(d, 0))
    T5 = syn.frames_for_seconds(5.0, d.sample_rate, d.hop_length)
    mels = [torch.from_numpy(syn.make_mel(d.feat_dims, T5, 40 + i))[None] for i in range(8)]
    if warm:
        model.generate_many(mels, None, False, 11000, 550, True, seed=1)
    outs, dt = _timed(lambda: model.generate_many(mels, None, False, 11000, 550, True, seed=2))
    ms, L2 = model.loop_handle().elapsed_ms(), T5 * d.hop_length
    n = sum(o.shape[0] for o in outs)
    res["config2_8_streams"] = {"samples_per_s": n / dt, "rtf_per_gpu": n / dt / sr, "rtf_per_stream": n / 8 / dt / sr,
                                "rows": 8,
                                "loop_steps": L2, "device_ms": ms, "wall_s": dt, "us_per_loop_step": ms * 1e3 / L2,
                                "kernel_path": model.loop_handle().info["last_path"],
                                "roofline": hbm_roofline(loop_weight_bytes(d) + 8 * COND_BYTES_PER_ROW_STEP, ms * 1e3 / L2,
                                                         "algorithmic bytes per step (all loop weights once + 836 B "
                                                         "per row) / step time; weights resident, latency-bound"),
                                "note": "8 independent 5 s utterances, unbatched, WaveRNN.generate_many (ONE launch of "
                                        "fatchord_xcd_kernel, one utterance per XCD); rate over the whole call "
                                        "(upsample, loop, float64 post)"}
    # serving throughput: 32 concurrent unbatched utterances (4 per XCD on the many-row MFMA kernel) —
    # per-stream latency traded for aggregate rate
    mels = [torch.from_numpy(syn.make_mel(d.feat_dims, T5, 140 + i))[None] for i in range(32)]
    if warm:
        model.generate_many(mels, None, False, 11000, 550, True, seed=1)
    outs, dt = _timed(lambda: model.generate_many(mels, None, False, 11000, 550, True, seed=2))
    ms = model.loop_handle().elapsed_ms()
    n = sum(o.shape[0] for o in outs)
    res["config2_32_streams"] = {"samples_per_s": n / dt, "rtf_per_gpu": n / dt / sr, "rtf_per_stream": n / 32 / dt / sr,
                                 "rows": 32, "loop_steps": L2, "device_ms": ms, "wall_s": dt,
                                 "us_per_loop_step": ms * 1e3 / L2, "kernel_path": model.loop_handle().info["last_path"],
                                 "roofline": hbm_roofline(loop_weight_bytes(d) + 32 * COND_BYTES_PER_ROW_STEP,
                                                          ms * 1e3 / L2, "as config2_8_streams"),
                                 "note": "32 independent 5 s utterances, unbatched (batch-1 streams), one "
                                         "WaveRNN.generate_many launch of fatchord_xcdm_kernel (4 rows per XCD): "
                                         "aggregate serving rate over the whole call"}
    del model
    # config 1's model (RAW 9-bit, rnn 512) on the GPU through the drop-in generate(): 1 s unbatched
    # (the reference runs it on the CPU) and a 5 s utterance fold-batched
    dr = syn.DEFAULT_RAW
    model = _mol_model(dr, dev, syn.make_fatchord_state(dr, 0))
    for key, sec, batched in (("config1_raw_1s_unbatched", 1.0, False), ("config1_raw_5s_fold_batched", 5.0, True)):
        mel = torch.from_numpy(syn.make_mel(dr.feat_dims, syn.frames_for_seconds(sec, dr.sample_rate, dr.hop_length),
                                            5))[None]
        if warm:
            model.generate(mel, None, batched, 11000, 550, True, seed=1, verbose=False)
        out, dt = _timed(lambda: model.generate(mel, None, batched, 11000, 550, True, seed=2, verbose=False))
        h = model.loop_handle()
        res[key] = {"samples_per_s": out.shape[0] / dt, "rtf": out.shape[0] / dt / dr.sample_rate, "wall_s": dt,
                    "device_ms": h.elapsed_ms(), "kernel_path": h.info["last_path"],
                    "note": "RAW 9-bit (bits mode, mu-law) generate() of a synthetic mel on the drop-in; path 7 = "
                            "fatchord_xcdm_kernel's softmax head; rate over the whole generate() wall time"}
    del model
    # config 3
    state3 = syn.make_fatchord_state(d, 0)
    model = _mol_model(d, dev, state3)
    mel = torch.from_numpy(syn.make_mel(d.feat_dims, syn.frames_for_seconds(60.0, d.sample_rate, d.hop_length), 3))[None]
    if warm:
        model.generate(mel, None, True, 11000, 550, True, seed=1, verbose=False)     # MIOpen tunes per shape
    out, dt = _timed(lambda: model.generate(mel, None, True, 11000, 550, True, seed=2, verbose=False))
    ms = model.loop_handle().elapsed_ms()
    flops = 2.0 * MOL_MACS_PER_ROW_STEP * 115 * 12100
    res["config3_mol_fold_60s"] = {"samples_per_s": out.shape[0] / dt, "rtf": out.shape[0] / dt / d.sample_rate,
                                   "rows": 115, "loop_steps": 12100, "device_ms": ms, "wall_s": dt,
                                   "us_per_loop_step": ms * 1e3 / 12100,
                                   "kernel_path": model.loop_handle().info["last_path"],
                                   "roofline": {"bound": "fp32 (vector/mfma)", "achieved": flops / (ms / 1e3) / 1e12,
                                                "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                                                "frac": flops / (ms / 1e3) / 1e12 / FP32_PEAK_TFLOPS,
                                                "note": "algorithmic FLOP = 2 x 3 825 152 MAC x 115 rows per step "
                                                        "(SURVEY.md 8(d): AI 57 F/B > ridge); device time of the loop "
                                                        "launches incl. the terms GEMMs between time chunks"}}
    if cpu_steps > 0:
        from oracle import torch_cpu
        n = min(cpu_steps, 12100)
        noise = syn.make_noise("MOL", 115, 12100, d.n_classes, 7)
        r = torch_cpu.timed_generate(state3, d, mel[0].numpy(), True, 11000, 550, True, noise, loop_steps=n,
                                     threads=threads)
        t_cpu = r["loop_s"] + n / 12100 * (r["pre_s"] + r["post_s"])
        res["config3_mol_fold_60s"]["cpu_baseline"] = {
            "value": n * 115 / t_cpu, "unit": "samples/s", "cores": r["threads"], "kind": "port",
            "rtf": n * 115 / t_cpu / sr, "loop_s": r["loop_s"], "pre_s": r["pre_s"], "post_s": r["post_s"],
            "sample": f"PyTorch-CPU eager fold-batched generate() (oracle/torch_cpu.py, {r['threads']} threads): "
                      f"upsample + fold of the whole 60 s mel, {n} of 12100 loop steps x 115 folds, float64 post of "
                      f"the whole utterance; value = loop-step samples / (loop time + {n / 12100:.3f} x pre/post)"}
    del model
    return res


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _timed_ranks(fn, world: int, dev):
    """fn() between barrier + synchronize pairs on every rank; (result, max elapsed over ranks)."""
    _sync(dev)
    if world > 1:
        dist.barrier()
    t = time.perf_counter()
    out = fn()
    _sync(dev)
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return out, float(el[0])


def _max_over_ranks(x: float, world: int, dev) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


UTT4_PER_RANK, UTT5_PER_RANK, L5 = 8, 32, 16000


def _config4_record(outs, dt, ms, world, L4, info) -> dict:
    n4 = UTT4_PER_RANK * world
    n = sum(o.shape[0] for o in outs)
    return {
        "samples_per_s": n / dt, "rtf": n / dt / 22050, "rtf_per_gpu": n / dt / 22050 / world,
        "utterances": n4, "n_gpus": world, "rows_per_gpu": UTT4_PER_RANK, "loop_steps": L4,
        "device_ms": ms, "wall_s": dt, "us_per_loop_step": ms * 1e3 / L4,
        "loop_samples_per_s": n4 * L4 / ms * 1e3,
        "sparse_blocks_per_gate_row": info["sparse_blocks"], "kernel_path": info["last_path"],
        "roofline": hbm_roofline(SPARSE896_BYTES_PER_STEP + UTT4_PER_RANK * COND_BYTES_PER_ROW_STEP, ms * 1e3 / L4,
                                 "SURVEY.md 8(d) bytes per step (sparse weights + int16 block indices once + "
                                 "836 B per row) / step time of the slowest rank's launch; blocks resident, "
                                 "latency-bound"),
        "note": f"{n4} synthetic 5 s mels through sharding.generate_sharded over {world} GPU(s): each rank runs "
                "its 8 as ONE launch of fatchord_xcds_kernel (path 6, one utterance per XCD), the audio is "
                "all-gathered to rank 0; samples_per_s = all utterances' samples / max-over-ranks wall time "
                "(MelResNet + upsample, loop incl. the conditioning terms, post, gather)"}


def _config5_record(outs, dt, ms, world, info) -> dict:
    n5 = UTT5_PER_RANK * world
    n = sum(o.size for o in outs)
    return {
        "samples_per_s": n / dt, "rtf": n / dt / 16000.0, "rtf_per_gpu": n / dt / 16000.0 / world,
        "utterances": n5, "n_gpus": world, "rows_per_gpu": UTT5_PER_RANK, "loop_steps": L5,
        "device_ms": ms, "wall_s": dt, "us_per_loop_step": ms * 1e3 / L5,
        "loop_samples_per_s": n5 * L5 / ms * 1e3, "kernel_path": info["last_path"],
        "roofline": hbm_roofline(DM_BYTES_PER_STEP + 4 * UTT5_PER_RANK, ms * 1e3 / L5,
                                 "SURVEY.md 8(d) bytes per step (weights once + 4 B per row) / step time of the "
                                 "slowest rank's launch; weights resident in each XCD's registers + LDS (path 8 = "
                                 "deepmind_xcd_kernel, 4 rows per XCD), hand-off-latency-bound"),
        "note": f"{n5} utterances of 16000 samples through sharding.generate_sharded_deepmind over {world} GPU(s) "
                "(32 rows per rank in one generate(batch=32) launch, outputs all-gathered to rank 0); rate over "
                "the max-over-ranks wall time incl. the label D2H and the gather"}


def sharded_configs(dev, world: int, rank: int, warm: bool = True, cpu_steps: int = 0, threads: int = 1,
                    stub: bool = False) -> dict:
    """BASELINE configs 4 and 5 as stated — utterance batches sharded over the GPUs of the node
    (`wavernn_amd.sharding`: contiguous blocks, one persistent launch per rank, the finished audio
    all-gathered to rank 0 over RCCL) — at 8 and 32 utterances PER RANK (weak scaling: at N = 8
    that is BASELINE's 64 and 256):
      4: rnn 896 with 95 % 4x4 block-sparse GRU weights, 5 s MoL utterances, unbatched
         (gen_wavernn.py:11-35 vocodes a list; generate_sharded);
      5: deepmind dual softmax, 1 s at 16 kHz (deepmind_version.py:75-165; generate_sharded_deepmind).
    Each leg is timed between barriers on every rank, elapsed = max over ranks, samples = all
    ranks'.  rank 0 returns the records (cpu_baseline beside each, timed after the legs).
    `stub`: no GPU — the same sharding, gather, timing and records around a stand-in generation
    (tests of the N > 1 contract on gloo ranks)."""
    from wavernn_amd import sharding
    res = {}
    d4 = syn.SPARSE896_MOL
    T5 = syn.frames_for_seconds(5.0, d4.sample_rate, d4.hop_length)
    L4 = T5 * d4.hop_length
    n4, n5 = UTT4_PER_RANK * world, UTT5_PER_RANK * world
    mels = [syn.make_mel(d4.feat_dims, T5, 60 + i)[None] for i in range(n4)]
    # ---- config 4
    if stub:
        model, state4 = None, None
        stub4 = lambda ii, ms, r0: [np.zeros((T5 - 1) * d4.hop_length) for _ in ii]   # noqa: E731
        one_row = type("OneRow", (), {"rows_of": staticmethod(lambda T, b, t, o: 1)})   # unbatched: 1 row each
        run4 = lambda seed: sharding.generate_sharded(one_row, mels, False, 11000, 550, True,  # noqa: E731
                                                      base_seed=seed, device=dev, generate_fn=stub4)
    else:
        from wavernn_amd.pruning import prune_state
        state4 = prune_state(syn.make_fatchord_state(d4, 0), 0.95)
        model = _mol_model(d4, dev, state4)
        run4 = lambda seed: sharding.generate_sharded(model, mels, False, 11000, 550, True,  # noqa: E731
                                                      base_seed=seed, device=dev)
    if warm:
        run4(1)
    outs, dt = _timed_ranks(lambda: run4(2), world, dev)
    info = {"sparse_blocks": 0, "last_path": 0} if stub else model.loop_handle().info
    ms = _max_over_ranks(dt * 1e3 if stub else model.loop_handle().elapsed_ms(), world, dev)
    if rank == 0:
        res["config4_sparse896_8utt"] = _config4_record(outs, dt, ms, world, L4, info)
    del model
    # ---- config 5
    dm = syn.DEFAULT_DM
    if stub:
        model, state5 = None, None
        run5 = lambda seed, L=L5: sharding.generate_sharded_deepmind(  # noqa: E731
            None, n5, L, base_seed=seed, device=dev, generate_fn=lambda ii, r0: [np.zeros(L) for _ in ii])
    else:
        from wavernn_amd.deepmind_version import WaveRNN as DeepmindWaveRNN
        state5 = syn.make_deepmind_state(dm, 0)
        model = DeepmindWaveRNN(**dm.ctor_kwargs()).to(dev)
        model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state5.items()})
        run5 = lambda seed, L=L5: sharding.generate_sharded_deepmind(model, n5, L, base_seed=seed,  # noqa: E731
                                                                     device=dev)
    if warm:
        run5(1, 100)
    outs5, dt = _timed_ranks(lambda: run5(2), world, dev)
    info = {"last_path": 0} if stub else model.loop_handle().info
    ms = _max_over_ranks(dt * 1e3 if stub else model.loop_handle().elapsed_ms(), world, dev)
    if rank == 0:
        res["config5_deepmind_32utt"] = _config5_record(outs5, dt, ms, world, info)
    del model
    if rank == 0 and cpu_steps > 0 and not stub:
        from oracle import torch_cpu
        n = min(cpu_steps, L4)
        noise = syn.make_noise("MOL", 1, n, d4.n_classes, 7)
        r = torch_cpu.timed_generate(state4, d4, mels[0][0], False, 11000, 550, True, noise, loop_steps=n,
                                     threads=threads)
        t_cpu = r["loop_s"] + n / L4 * (r["pre_s"] + r["post_s"])
        res["config4_sparse896_8utt"]["cpu_baseline"] = {
            "value": n / t_cpu, "unit": "samples/s", "cores": r["threads"], "kind": "port",
            "rtf": n / t_cpu / 22050, "loop_s": r["loop_s"], "pre_s": r["pre_s"], "post_s": r["post_s"],
            "sample": f"PyTorch-CPU eager generate() of ONE 5 s utterance as the reference vocodes a list "
                      f"(oracle/torch_cpu.py, {r['threads']} threads, the pruned weights as dense matrices): "
                      f"{n} of {L4} loop steps + {n / L4:.3f} x the pre/post time"}
        n = min(cpu_steps, L5)
        r = torch_cpu.timed_deepmind(state5, UTT5_PER_RANK, syn.make_dm_noise(UTT5_PER_RANK, n, dm.quantisation, 7),
                                     n, threads=threads)
        res["config5_deepmind_32utt"]["cpu_baseline"] = {
            "value": n * UTT5_PER_RANK / r["loop_s"], "unit": "samples/s", "cores": r["threads"], "kind": "port",
            "rtf": n * UTT5_PER_RANK / r["loop_s"] / 16000.0, "loop_s": r["loop_s"],
            "sample": f"PyTorch-CPU eager deepmind loop (oracle/torch_cpu.deepmind_loop: the reference's per-step "
                      f"ops for 32 rows at once, {r['threads']} threads), {n} of {L5} steps x 32 rows"}
    return res


def attach_traffic(rec: dict, traffic, traffic_from) -> None:
    """Per-config HBM bytes per loop step (PMC) beside each secondary line's roofline: the
    fold-batched line and every other_configs entry; null with the reason when unavailable."""
    lines = dict(rec.get("other_configs", {}))
    if "fold_batched" in rec:
        lines["fold_batched"] = rec["fold_batched"]
    for key, v in lines.items():
        if "roofline" not in v:
            continue
        tr = (traffic or {}).get("other_configs", {}).get(key)
        v["roofline"]["traffic_per_step"] = tr["bytes_per_step"] if tr is not None else None
        v["roofline"]["traffic_from"] = traffic_from


# ------------------------------------------------------------------------------- main
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=5.0, help="utterance length")
    ap.add_argument("--mode", default="MOL", choices=["MOL", "RAW"])
    ap.add_argument("--batched", action="store_true", help="fold-batched generate (target 11000, overlap 550)")
    ap.add_argument("--cpu-steps", type=int, default=25000, help="loop steps timed for cpu_baseline (0: skip)")
    ap.add_argument("--other-configs", type=int, default=1, help="also time BASELINE configs 1/3/4/5 on this GPU (N=1)")
    ap.add_argument("--fold-batched", type=int, default=1, help="also time the same utterance through generate(batched=True)")
    ap.add_argument("--pmc", type=int, default=1, help="live rocprofv3 FETCH_SIZE/WRITE_SIZE passes for roofline.traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stub", action="store_true",
                    help="no GPU: gloo ranks time a stand-in generation (tests of the launcher / timing contract)")
    return ap.parse_args(argv)


def timed_steps(step, steps: int, warmup: int, world: int, dev):
    """W untimed warm-up steps, then K steps between barrier + synchronize pairs; returns the
    elapsed time MAX over ranks and the samples SUMMED over ranks."""
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    for i in range(warmup):
        step(-1 - i)
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    n_samples = 0
    for i in range(steps):
        n_samples += step(i)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    tot = torch.tensor([float(n_samples)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    return float(stats[0]), float(tot[0])


def stub_main(args, world, rank):
    """The launcher + timing contract without a GPU: every rank 'generates' 22 050 samples per
    step (a 10 ms sleep) and rank 0 gathers them, as the real step does."""
    dev = torch.device("cpu")
    if world > 1:
        dist.init_process_group("gloo")
    from wavernn_amd import sharding

    def step(i):
        time.sleep(0.01)
        out = np.zeros(22050)
        if world > 1:
            sharding.gather_audio({rank: out}, world, dev)
        return out.shape[0]

    elapsed, total = timed_steps(step, args.steps, args.warmup, world, dev)
    sharded = sharded_configs(dev, world, rank, stub=True) if args.other_configs else {}
    if rank == 0:
        print(json.dumps({"metric": "stub", "value": total / elapsed, "unit": "samples/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                          "higher_is_better": True, "scaling": "weak", "data": "stub",
                          "other_configs": sharded}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one rank per GPU: two ranks' persistent launches cannot share a GPU (each needs every CU
        # co-resident), so refuse rather than time out (device_count() does not initialise the GPU)
        if not args.stub and torch.cuda.device_count() < args.gpus:
            sys.exit(f"bench.py --gpus {args.gpus}: only {torch.cuda.device_count()} GPU(s) visible")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub:
        return stub_main(args, world, rank)
    if args.pmc_child:
        args.steps, args.warmup, args.cpu_steps, args.fold_batched, args.pmc = 1, 0, 0, 0, 0
    # HBM traffic passes first, while this process has not touched the GPU (child processes)
    traffic, traffic_from = None, None
    headline_shape = not args.batched and args.mode == "MOL" and abs(args.seconds - 5.0) < 1e-9
    if rank == 0 and headline_shape and not args.pmc_child:
        # rank 0 only (its GPU = the children's cuda:0); the other ranks wait in the rendezvous
        live = pmc_live() if args.pmc else None
        traffic, traffic_from = resolve_traffic(live, PMC_PROFILE)

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # generous rendezvous timeout: rank 0 runs the PMC passes before it joins
        from datetime import timedelta
        dist.init_process_group("nccl", device_id=dev, timeout=timedelta(minutes=30))

    d = syn.DEFAULT_MOL if args.mode == "MOL" else syn.DEFAULT_RAW
    state = syn.make_fatchord_state(d, 0)
    model = _mol_model(d, dev, state)
    T = syn.frames_for_seconds(args.seconds, d.sample_rate, d.hop_length)
    mel = torch.from_numpy(syn.make_mel(d.feat_dims, T, seed=1 + rank))[None]
    target, overlap = 11000, 550
    loop_ms = []

    from wavernn_amd import sharding

    def step(i):
        # every rank vocodes its own utterance (Philox keyed by global row = i·world + rank);
        # the finished audio is gathered to rank 0 — the path's only collective
        g = i * world + rank
        out = model.generate(mel, None, args.batched, target, overlap, True, seed=1000, row_offset=g, verbose=False)
        if world > 1:
            sharding.gather_audio({rank: out}, world, dev)
        if i >= 0:
            loop_ms.append(model.loop_handle().elapsed_ms())
        return out.shape[0]

    elapsed, total_samples = timed_steps(step, args.steps, args.warmup, world, dev)
    lm = torch.tensor([float(np.mean(loop_ms))], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(lm, op=dist.ReduceOp.MAX)
    loop_ms_max = float(lm[0])

    if args.pmc_child:
        # the same order tools/pmc_summary.py attributes dispatches in: headline, fold-batched,
        # then the other configs
        model.generate(mel, None, True, target, overlap, True, seed=7, verbose=False)
        other_configs(dev, warm=False)
        sharded_configs(dev, 1, 0, warm=False)
        return

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    # configs 4 / 5 as BASELINE states them: utterance batches sharded over all ranks (collective legs:
    # every rank takes part; rank 0 gets the records, with their CPU baselines timed after the legs)
    sharded = {}
    if args.other_configs and args.mode == "MOL":
        sharded = sharded_configs(dev, world, rank, cpu_steps=min(args.cpu_steps, 2000), threads=threads)

    if rank == 0:
        cond, _ = model.conditioning(mel, args.batched, target, overlap)
        L, B, _ = cond.shape
        wbytes = loop_weight_bytes(d)
        bytes_per_launch = L * (wbytes + B * COND_BYTES_PER_ROW_STEP)
        achieved = bytes_per_launch / (loop_ms_max / 1e3) / 1e9
        value = total_samples / elapsed
        info = model.loop_handle().info
        rec = {
            "metric": "audio samples/sec/GPU (22.05 kHz MoL, rnn_dims=512) + real-time factor at batch=1"
            if args.mode == "MOL" else "audio samples/sec (22.05 kHz RAW 9-bit, rnn_dims=512)",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic mel (seeded uniform [0,1)), random weights of the 800k MoL architecture",
            "config": {
                "workload": f"fatchord WaveRNN {args.mode} generate(), {args.seconds:g} s utterance per GPU, "
                            f"{'fold-batched target 11000/overlap 550' if args.batched else 'unbatched (batch=1)'}",
                "mode": args.mode, "rnn_dims": d.rnn_dims, "fc_dims": d.fc_dims, "utterance_s": args.seconds,
                "loop_steps": L, "rows": B, "samples_per_utterance": int(total_samples / args.steps / world),
                "parallelism": f"utterance-sharded x{world}",
                "kernel": KERNELS.get(info["last_path"], str(info["last_path"])),
            },
            "rtf_per_gpu": value / world / d.sample_rate,
            "loop_kernel_ms": loop_ms_max,
            "us_per_loop_step": loop_ms_max * 1e3 / L,
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic["bytes"] if traffic else None,
                "traffic_from": traffic_from,
                "note": "achieved = algorithmic bytes (all loop weights fp32 per step + 836 B/row-step) per launch "
                        "/ launch time (HIP events); the weights are LDS/VGPR-resident on one XCD's 32 CUs "
                        "(fatchord_xcd_kernel), the kernel is hand-off-latency bound. traffic = 2 x FETCH_SIZE + "
                        "WRITE_SIZE bytes of the headline launch (gfx950 read correction; traffic_from says where "
                        "it came from, null when the live passes failed): conditioning-terms reads; the "
                        "hand-offs stay in the XCD's L2",
            },
        }
        if args.fold_batched and not args.batched and args.mode == "MOL":
            # the same utterance through the reference's default generate() mode
            # (hparams voc_gen_batched = True: 11000/550 folds, one multi-row launch)
            model.generate(mel, None, True, target, overlap, True, seed=7, verbose=False)
            outb, dtb = _timed(lambda: model.generate(mel, None, True, target, overlap, True, seed=8, verbose=False))
            kb = model.loop_handle().elapsed_ms()
            condb, _ = model.conditioning(mel, True, target, overlap)
            usb = kb * 1e3 / condb.shape[0]
            rec["fold_batched"] = {
                "samples_per_s": outb.shape[0] / dtb, "rtf": outb.shape[0] / dtb / d.sample_rate,
                "rows": int(condb.shape[1]), "loop_steps": int(condb.shape[0]), "device_ms": kb,
                "us_per_loop_step": usb,
                "kernel_path": model.loop_handle().info["last_path"],
                "kernel": KERNELS.get(model.loop_handle().info["last_path"]),
                "roofline": hbm_roofline(wbytes + int(condb.shape[1]) * COND_BYTES_PER_ROW_STEP, usb,
                                         "algorithmic bytes per step (all loop weights once + 836 B per row) / step "
                                         "time of the launch; weights resident as MFMA operands, latency-bound"),
                "note": "same 5 s utterance, generate(batched=True) as gen_wavernn.py runs it with the 800k "
                        "hparams (10 folds in one launch) + conditioning-terms GEMM; rate over the whole "
                        "generate() wall time (upsample, loop, float64 post)",
            }
        if args.other_configs and args.mode == "MOL":
            # single-GPU configs (1, 2 x 8 streams, 3) on rank 0's GPU, then the sharded legs' records
            rec["other_configs"] = other_configs(dev, cpu_steps=min(args.cpu_steps, 2000), threads=threads)
            rec["other_configs"].update(sharded)
        attach_traffic(rec, traffic, traffic_from)
        if args.cpu_steps > 0:
            # the reference's op sequence on this host's cores: PyTorch-CPU eager (oracle/torch_cpu.py),
            # whole pre/post + a bounded slice of the loop; and the C oracle on the same slice
            from oracle import oracle, torch_cpu
            n = min(args.cpu_steps, L)
            noise = syn.make_noise(d.mode, B, L, d.n_classes, 7)
            r = torch_cpu.timed_generate(state, d, mel[0].numpy(), args.batched, target, overlap, True, noise,
                                         loop_steps=n, threads=threads)
            frac = n / L
            t_cpu = r["loop_s"] + frac * (r["pre_s"] + r["post_s"])
            rec["cpu_baseline"] = {
                "value": n * B / t_cpu, "unit": "samples/s", "cores": r["threads"], "kind": "port",
                "sample": f"PyTorch-CPU eager generate() (oracle/torch_cpu.py, torch.set_num_threads({r['threads']})): "
                          f"upsample + fold of the whole {args.seconds:g} s mel, {n} of {L} loop steps x {B} row(s), "
                          f"float64 post-processing of the whole utterance; value = loop-step samples / (loop time + "
                          f"{frac:.3f} x pre/post time)",
                "loop_s": r["loop_s"], "pre_s": r["pre_s"], "post_s": r["post_s"],
                "rtf": n * B / t_cpu / d.sample_rate}
            cpu = cond.transpose(0, 1).cpu().numpy()
            mels_c = np.ascontiguousarray(cpu[:, :n, :d.feat_dims])
            aux_c = np.ascontiguousarray(cpu[:, :n, d.feat_dims:])
            oracle.build()
            t = time.perf_counter()
            oracle.fatchord_loop(state, d.mode, mels_c, aux_c, noise[:n])
            dt = time.perf_counter() - t
            rec["cpu_baseline_c_oracle"] = {"value": n * B / dt, "unit": "samples/s", "cores": 1, "kind": "port",
                                            "sample": f"{n} of {L} loop steps x {B} row(s), same weights/conditioning, "
                                                      f"C oracle (oracle/wavernn_oracle.c, gcc -O3, 1 thread), loop only",
                                            "seconds": dt}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
