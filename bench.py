"""Headline benchmark: WaveRNN MoL (rnn_dims 512) generation on MI355X.

Workload (BASELINE.json configs[1]): one 5 s utterance per GPU (synthetic 80-band mel,
T = 401 frames → 110 275 loop steps, 110 000 output samples), unbatched (batch = 1), MoL
sampling, random weights of the 800k-step MoL architecture (hparams.py).  A "step" of this
benchmark is one full `WaveRNN.generate()` of that utterance (upsample → persistent HIP
loop → float64 post-processing).  N GPUs = N ranks, one utterance each (weak scaling; the
utterances are independent, there is no collective in the data path).

Prints ONE JSON line on rank 0.  `roofline` is computed for the persistent loop kernel from
HIP events around its launch; `cpu_baseline` times the reference's own op sequence as a
PyTorch-CPU eager restatement (oracle/torch_cpu.py: upsample, the per-step loop, float64 post) on
this host's cores over a bounded slice of the same workload; `cpu_baseline_c_oracle` the
single-threaded C oracle (oracle/wavernn_oracle.c) on the same slice.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
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
PMC_PROFILE = os.environ.get("WRNN_PMC_PROFILE", os.path.join(REPO, "profiles", "r03_v7_pmc_traffic.json"))
SPARSE896_BYTES_PER_STEP = 5536598   # config 4 sparse values + int16 block indices, fp32
DM_BYTES_PER_STEP = 12200196         # config 5 deepmind weights, fp32


def pmc_traffic_bytes(mode: str, batched: bool, seconds: float):
    """HBM-side bytes per launch from the committed rocprofv3 PMC passes (FETCH_SIZE +
    WRITE_SIZE, separate passes) for this exact workload, or None.  gfx950 correction
    (MI355X_MICROARCH.md): FETCH_SIZE counts half the bytes of 16-B-per-lane reads."""
    if mode != "MOL" or batched or abs(seconds - 5.0) > 1e-9 or not os.path.exists(PMC_PROFILE):
        return None
    c = json.load(open(PMC_PROFILE))["counters"]
    return 1024.0 * (2.0 * c["FETCH_SIZE"]["value_kib"] + c["WRITE_SIZE"]["value_kib"])


def pmc_config_traffic(key: str):
    """HBM bytes per loop step of another config's loop kernel from the same PMC passes, or None."""
    if not os.path.exists(PMC_PROFILE):
        return None
    c = json.load(open(PMC_PROFILE)).get("other_configs", {}).get(key)
    return c["bytes_per_step"] if c else None
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


def other_configs(dev) -> dict:
    """BASELINE configs 3-5 on one GPU (synthetic inputs, random weights of each architecture):
      3: MoL fold-batched generate() of one 60 s utterance (115 folds x 12 100 steps);
      4: rnn 896 with 95 % 4x4 block-sparse GRU weights, 8 utterances of 5 s (8 rows) per GPU;
      5: deepmind dual softmax, 32 utterances of 1 s at 16 kHz (32 rows) per GPU;
    plus the headline architecture serving 8 independent batch-1 streams at once (one per XCD)."""
    from wavernn_amd.fatchord_version import WaveRNN
    from wavernn_amd.loop import DeepmindLoop, FatchordLoop
    from wavernn_amd.pruning import prune_state
    res = {}
    # config 2 architecture, 8 concurrent unbatched utterances (per-stream latency unchanged)
    d = syn.DEFAULT_MOL
    L2, B2 = syn.frames_for_seconds(5.0, d.sample_rate, d.hop_length) * d.hop_length, 8
    loop = FatchordLoop(d.mode, d.rnn_dims, d.fc_dims, d.aux_dims, d.feat_dims, d.n_classes)
    loop.set_weights(syn.make_fatchord_state(d, 0))
    mels, aux = syn.make_conditioning(B2, L2, d.feat_dims, d.res_out_dims, 4)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(dev)
    loop.generate(cond[:100].contiguous(), seed=1)
    loop.generate(cond, seed=2)
    ms = loop.elapsed_ms()
    res["config2_8_streams"] = {"samples_per_s": B2 * L2 / ms * 1e3, "rtf_per_stream": L2 / ms * 1e3 / d.sample_rate,
                                "rows": B2, "loop_steps": L2, "device_ms": ms, "us_per_loop_step": ms * 1e3 / L2,
                                "kernel_path": loop.info["last_path"],
                                "roofline": hbm_roofline(loop_weight_bytes(d) + B2 * COND_BYTES_PER_ROW_STEP, ms * 1e3 / L2,
                                                         "algorithmic bytes per step (all loop weights once + 836 B "
                                                         "per row) / step time; weights resident, latency-bound"),
                                "note": "8 independent 5 s utterances, unbatched, one per XCD in one launch of "
                                        "fatchord_xcd_kernel (path 5), from upsampled conditioning (upsample "
                                        "excluded), incl. the conditioning-terms GEMM"}
    del cond
    loop.close()
    # config 1's model (RAW 9-bit, rnn 512) on the GPU through the drop-in generate(): 1 s unbatched
    # (the reference runs it on the CPU) and a 5 s utterance fold-batched
    dr = syn.DEFAULT_RAW
    model = WaveRNN(**dr.ctor_kwargs()).to(dev)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(dr, 0).items()})
    for key, sec, batched in (("config1_raw_1s_unbatched", 1.0, False), ("config1_raw_5s_fold_batched", 5.0, True)):
        mel = torch.from_numpy(syn.make_mel(dr.feat_dims, syn.frames_for_seconds(sec, dr.sample_rate, dr.hop_length),
                                            5))[None]
        model.generate(mel, None, batched, 11000, 550, True, seed=1, verbose=False)
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = model.generate(mel, None, batched, 11000, 550, True, seed=2, verbose=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        h = model.loop_handle()
        ms = h.elapsed_ms()
        res[key] = {"samples_per_s": out.shape[0] / dt, "rtf": out.shape[0] / dt / dr.sample_rate, "wall_s": dt,
                    "device_ms": ms, "kernel_path": h.info["last_path"],
                    "note": "RAW 9-bit (bits mode, mu-law) generate() of a synthetic mel on the drop-in; path 7 = "
                            "fatchord_xcdm_kernel's softmax head; rate over the whole generate() wall time"}
    del model
    # config 3
    d = syn.DEFAULT_MOL
    model = WaveRNN(**d.ctor_kwargs()).to(dev)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in syn.make_fatchord_state(d, 0).items()})
    mel = torch.from_numpy(syn.make_mel(d.feat_dims, syn.frames_for_seconds(60.0, d.sample_rate, d.hop_length), 3))[None]
    model.generate(mel, None, True, 11000, 550, True, seed=1, verbose=False)     # warm (MIOpen tunes per shape)
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = model.generate(mel, None, True, 11000, 550, True, seed=2, verbose=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
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
    del model
    # config 4
    d4 = syn.SPARSE896_MOL
    L4, B4 = syn.frames_for_seconds(5.0, d4.sample_rate, d4.hop_length) * d4.hop_length, 8
    loop = FatchordLoop(d4.mode, d4.rnn_dims, d4.fc_dims, d4.aux_dims, d4.feat_dims, d4.n_classes)
    loop.set_weights(prune_state(syn.make_fatchord_state(d4, 0), 0.95))
    mels, aux = syn.make_conditioning(B4, L4, d4.feat_dims, d4.res_out_dims, 4)
    cond = torch.from_numpy(np.concatenate([mels, aux], 2).transpose(1, 0, 2).copy()).to(dev)
    loop.generate(cond[:100].contiguous(), seed=1)
    ms = 0.0
    loop.generate(cond, seed=2)
    ms = loop.elapsed_ms()
    res["config4_sparse896_8utt"] = {"samples_per_s": B4 * L4 / ms * 1e3, "rtf": B4 * L4 / ms * 1e3 / d4.sample_rate,
                                     "rows": B4, "loop_steps": L4, "device_ms": ms, "us_per_loop_step": ms * 1e3 / L4,
                                     "sparse_blocks_per_gate_row": loop.info["sparse_blocks"],
                                     "kernel_path": loop.info["last_path"],
                                     "roofline": hbm_roofline(SPARSE896_BYTES_PER_STEP + B4 * COND_BYTES_PER_ROW_STEP,
                                                              ms * 1e3 / L4,
                                                              "SURVEY.md 8(d) bytes per step (sparse weights + int16 "
                                                              "block indices once + 836 B per row) / step time; "
                                                              "blocks resident, latency-bound"),
                                     "note": "loop launch from upsampled conditioning (upsample excluded); path 6 = "
                                             "fatchord_xcds_kernel (one utterance per XCD, block-sparse GRU blocks), "
                                             "incl. the conditioning-terms GEMM"}
    loop.close()
    # config 5
    dm = syn.DEFAULT_DM
    B5, L5 = 32, 16000
    loop5 = DeepmindLoop(dm.hidden_size, dm.quantisation)
    loop5.set_weights(syn.make_deepmind_state(dm, 0))
    loop5.generate(B5, 100, seed=1)
    loop5.generate(B5, L5, seed=2)
    ms = loop5.elapsed_ms()
    res["config5_deepmind_32utt"] = {"samples_per_s": B5 * L5 / ms * 1e3, "rtf": B5 * L5 / ms * 1e3 / 16000.0,
                                     "rows": B5, "loop_steps": L5, "device_ms": ms, "us_per_loop_step": ms * 1e3 / L5,
                                     "kernel_path": loop5.info["last_path"],
                                     "roofline": hbm_roofline(DM_BYTES_PER_STEP + 4 * B5, ms * 1e3 / L5,
                                                              "SURVEY.md 8(d) bytes per step (weights once + 4 B per "
                                                              "row) / step time; weights resident in each XCD's "
                                                              "registers + LDS (path 8 = deepmind_xcd_kernel, 4 rows "
                                                              "per XCD), hand-off-latency-bound")}
    loop5.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=5.0, help="utterance length")
    ap.add_argument("--mode", default="MOL", choices=["MOL", "RAW"])
    ap.add_argument("--batched", action="store_true", help="fold-batched generate (target 11000, overlap 550)")
    ap.add_argument("--cpu-steps", type=int, default=25000, help="loop steps timed for cpu_baseline (0: skip)")
    ap.add_argument("--other-configs", type=int, default=1, help="also time BASELINE configs 3/4/5 on this GPU (N=1)")
    ap.add_argument("--fold-batched", type=int, default=1, help="also time the same utterance through generate(batched=True)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from wavernn_amd.fatchord_version import WaveRNN
    d = syn.DEFAULT_MOL if args.mode == "MOL" else syn.DEFAULT_RAW
    state = syn.make_fatchord_state(d, 0)
    model = WaveRNN(**d.ctor_kwargs()).to(dev)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
    T = syn.frames_for_seconds(args.seconds, d.sample_rate, d.hop_length)
    mel = torch.from_numpy(syn.make_mel(d.feat_dims, T, seed=1 + rank))[None]
    target, overlap = 11000, 550

    from wavernn_amd import sharding

    def step(i):
        # every rank vocodes its own utterance (global index = i·world + rank, Philox keyed by
        # it); the finished audio is gathered to rank 0 — the path's only collective
        g = i * world + rank
        out = model.generate(mel, None, args.batched, target, overlap, True, seed=1000 + g, verbose=False)
        if world > 1:
            sharding.gather_audio({rank: out}, world, dev)
        return out

    for i in range(args.warmup):
        step(-1 - i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    loop_ms = []
    t0 = time.perf_counter()
    n_samples = 0
    for i in range(args.steps):
        out = step(i)
        n_samples += out.shape[0]
        loop_ms.append(model.loop_handle().elapsed_ms())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = torch.tensor([elapsed, float(np.mean(loop_ms))], dtype=torch.float64, device=dev)
    tot = torch.tensor([float(n_samples)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed, loop_ms_max = float(stats[0]), float(stats[1])
    total_samples = float(tot[0])

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
                "loop_steps": L, "rows": B, "samples_per_utterance": int(n_samples / args.steps),
                "parallelism": f"utterance-sharded x{world}",
                "kernel": KERNELS.get(info["last_path"], str(info["last_path"])),
            },
            "rtf_per_gpu": value / world / d.sample_rate,
            "loop_kernel_ms": loop_ms_max,
            "us_per_loop_step": loop_ms_max * 1e3 / L,
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": pmc_traffic_bytes(args.mode, args.batched, args.seconds),
                "traffic_from": os.path.relpath(PMC_PROFILE, REPO) if pmc_traffic_bytes(args.mode, args.batched,
                                                                                       args.seconds) else None,
                "note": "achieved = algorithmic bytes (all loop weights fp32 per step + 836 B/row-step) per launch "
                        "/ launch time (HIP events); the weights are LDS/VGPR-resident on one XCD's 32 CUs "
                        "(fatchord_xcd_kernel), the kernel is hand-off-latency bound. "
                        f"traffic = 2 x FETCH_SIZE + WRITE_SIZE bytes per launch (gfx950 read correction), NOT measured "
                        f"in this run: read from the committed rocprofv3 --pmc passes of the same command in "
                        f"{os.path.relpath(PMC_PROFILE, REPO)} (traffic_from): conditioning-terms reads; the hand-offs "
                        f"stay in the XCD's L2",
            },
        }
        if args.fold_batched and not args.batched and args.mode == "MOL":
            # the same utterance through the reference's default generate() mode
            # (hparams voc_gen_batched = True: 11000/550 folds, one multi-row launch)
            model.generate(mel, None, True, target, overlap, True, seed=7, verbose=False)
            torch.cuda.synchronize()
            tb = time.perf_counter()
            outb = model.generate(mel, None, True, target, overlap, True, seed=8, verbose=False)
            torch.cuda.synchronize()
            dtb = time.perf_counter() - tb
            kb = model.loop_handle().elapsed_ms()
            condb, _ = model.conditioning(mel, True, target, overlap)
            rec["fold_batched"] = {
                "samples_per_s": outb.shape[0] / dtb, "rtf": outb.shape[0] / dtb / d.sample_rate,
                "rows": int(condb.shape[1]), "loop_steps": int(condb.shape[0]), "device_ms": kb,
                "us_per_loop_step": kb * 1e3 / condb.shape[0],
                "kernel_path": model.loop_handle().info["last_path"],
                "kernel": KERNELS.get(model.loop_handle().info["last_path"]),
                "note": "same 5 s utterance, generate(batched=True) as gen_wavernn.py runs it with the 800k "
                        "hparams (10 folds in one launch) + conditioning-terms GEMM; rate over the whole "
                        "generate() wall time (upsample, loop, float64 post)",
            }
        if args.other_configs and world == 1 and args.mode == "MOL":
            rec["other_configs"] = other_configs(dev)
            for key, v in rec["other_configs"].items():
                tr = pmc_config_traffic(key)
                if tr is not None and "roofline" in v:
                    v["roofline"]["traffic_per_step"] = tr   # HBM bytes per loop step (PMC, corrected)
        if args.cpu_steps > 0 and world == 1:
            # the reference's op sequence on this host's cores: PyTorch-CPU eager (oracle/torch_cpu.py),
            # whole pre/post + a bounded slice of the loop; and the C oracle on the same slice
            from oracle import oracle, torch_cpu
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
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
