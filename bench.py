#!/usr/bin/env python
"""DS2 training throughput on MI355X: audio-seconds/sec, 5xBiGRU-800, 32 x 10 s per GPU.

python bench.py [--gpus N --steps K --warmup W]          (N=1: plain process)
python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = the reference's train_batch (train.py:555-632) on the HIP path:
forward (conv/BN/5 BiGRU/FC/softmax), greedy decode + per-batch CER/WER, CTC (+grad), backward,
bucketed RCCL gradient all-reduce overlapped with backward (N > 1), clip 100 +
SGD-Nesterov.  Synthetic 10 s spectrograms [32, 1, 161, 1001] resident in HBM,
random-init weights (seed 123456), 150-label targets.  Weak scaling: 32
utterances per GPU.  Rank 0 prints one JSON line: ``value`` from the wall clock around
exactly K steps (the contract; max over ranks), plus the median per-step time from HIP
events (5 warm-up, median of 20).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

LABELS = "_'ABCDEFGHIJKLMNOPQRSTUVWXYZ2 "
CONF = dict(sample_rate=16000, window_size=0.02, window_stride=0.01, window='hamming')
BATCH, T_FRAMES, SECONDS, HIDDEN, LAYERS, LABEL_LEN = 32, 1001, 10.0, 800, 5, 150
# fp32 algorithmic work per training step at this shape (BASELINE.md §3 / SURVEY §8d)
TRAIN_FLOP_PER_STEP = 4.940e12
PEAK_F32_MFMA_TFLOPS = 157.3     # MI355X dense fp32 (MI355X_MICROARCH.md)
# fp32 GEMMs run as bf16x6 split products on the bf16 matrix cores (gemm.hip sxgemm2_kernel,
# fp32-accurate): their peak is the dense bf16 MFMA peak (16 x fp32) / 6 products
PEAK_BF16_MFMA_TFLOPS = 16 * PEAK_F32_MFMA_TFLOPS
PEAK_X6_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6


PEAK_H3_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 3
# the rate a bare MFMA loop reaches at the GEMM's own wave tile (2 x 10 16x16 tiles, 8 waves,
# fragments re-read from LDS every k-step, random operands, the clock the chip holds under
# it): scripts/mfma_ceiling.hip, profiles/r5b_mfma_ceiling.jsonl (fp32-equivalent TFLOP/s)
MEASURED_CEILING = {"x6": 300.0, "h3": 521.3}
CEILING_SOURCE = "profiles/r5b_mfma_ceiling.jsonl"


def gemm_mode():
    if os.environ.get("DS2_GEMM_X6", "1")[:1] == "0":
        return "fp32"
    return "x6" if os.environ.get("DS2_GEMM_H3", "1")[:1] == "0" else "h3"


def gemm_peak():
    """(peak TFLOP/s, arithmetic) of ds2_sgemm_ws as configured: the fp16x3 kernel by default,
    DS2_GEMM_H3=0 the bf16x6 kernel, DS2_GEMM_X6=0 fp32 MFMA."""
    mode = gemm_mode()
    if mode == "fp32":
        return PEAK_F32_MFMA_TFLOPS, "fp32 MFMA (v_mfma_f32_16x16x4_f32)"
    if mode == "h3":
        return PEAK_H3_TFLOPS, ("fp32 operands scaled per row by 2^e and split into 2 fp16 "
                                "terms, 3 products on v_mfma_f32_16x16x32_f16, fp32 accumulation "
                                "(fp16 dense peak / 3)")
    return PEAK_X6_TFLOPS, ("fp32 operands split into 3 bf16 terms, 6 products on "
                            "v_mfma_f32_16x16x32_bf16 (32x32x16 for a K tail), fp32 "
                            "accumulation (bf16 dense peak / 6)")


def _env_on(name: str) -> bool:
    return os.environ.get(name, "1")[:1] != "0"


def gru_fwd_kernel(x6f: bool):
    """(peak, arithmetic, kernel name) of the GRU forward recurrence as configured: fp16x3 by
    default (gru_split.hip), bf16x6 with DS2_GRU_H3=0, the fp32-MFMA kernel with
    DS2_GRU_X6=0."""
    if x6f and _env_on("DS2_GRU_H3") and _env_on("DS2_GRU_XL"):
        return (PEAK_H3_TFLOPS, "W_hh contraction, fp16x3 (fp32-accurate: per-row scaled fp16 "
                "hi/lo, the 8 samples' hi and lo stacked in one 16-row fragment: 2 "
                "v_mfma_f32_16x16x32_f16 per k-step and column tile), XCD-local groups of "
                "32-unit x 8-sample workgroups (gru_xl.hip)", "gru_fwd_xl_kernel")
    if x6f and _env_on("DS2_GRU_H3"):
        return (PEAK_H3_TFLOPS, "W_hh contraction, fp16x3 (fp32-accurate: per-row scaled fp16 "
                "hi/lo, 3 products) on v_mfma_f32_16x16x32_f16", "gru_fwd_x6_kernel")
    if x6f:
        return (PEAK_X6_TFLOPS, "W_hh contraction, bf16x6 (fp32-accurate) on "
                "v_mfma_f32_16x16x32_bf16", "gru_fwd_x6_kernel")
    return PEAK_F32_MFMA_TFLOPS, "W_hh contraction, fp32 MFMA", "gru_fwd_dop_kernel"


def gru_bwd_kernel(x6f: bool):
    """(peak, arithmetic, kernel name) of the GRU backward recurrence as configured: fp16x3
    records by default (gru_bwd_h3_kernel), the pre-split bf16x6 kernel with DS2_GRU_H3_BWD=0,
    the fp32-MFMA kernel with DS2_GRU_X6=0."""
    if x6f and _env_on("DS2_GRU_H3_BWD") and _env_on("DS2_GRU_XL"):
        return (PEAK_H3_TFLOPS, "W_hh^T contraction, fp16x3 (one record of stacked per-row "
                "scaled fp16 hi/lo fragments per producer and step; 4 v_mfma_f32_16x16x32_f16 "
                "per gate and 16 columns), XCD-local groups of 32-unit x 8-sample workgroups "
                "(gru_xl.hip)", "gru_bwd_xl_kernel")
    if x6f and _env_on("DS2_GRU_H3_BWD"):
        return (PEAK_H3_TFLOPS, "W_hh^T contraction, fp16x3 (one per-row scaled fp16 hi/lo "
                "record per producer and step) on v_mfma_f32_16x16x32_f16 / 16x16x16f16",
                "gru_bwd_h3_kernel")
    if x6f:
        return (PEAK_X6_TFLOPS, "W_hh^T contraction, bf16x6 (fp32-accurate, pre-split tiles) "
                "on v_mfma_f32_16x16x32_bf16", "gru_bwd_x6_kernel")
    return PEAK_F32_MFMA_TFLOPS, "W_hh^T contraction, fp32 MFMA (v_mfma_f32_16x16x4_f32)", "gru_bwd_dop_kernel"


def synthetic_batch(rank: int):
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.randn(BATCH, 1, 161, T_FRAMES, generator=g)
    tg = []
    for _ in range(BATCH):
        prev = -1
        for _ in range(LABEL_LEN):
            v = int(torch.randint(1, 29, (1,), generator=g))
            while v == prev:
                v = int(torch.randint(1, 29, (1,), generator=g))
            tg.append(v)
            prev = v
    targets = torch.tensor(tg, dtype=torch.int32)
    target_sizes = torch.full((BATCH,), LABEL_LEN, dtype=torch.int32)
    pct = torch.ones(BATCH)
    return x, targets, pct, target_sizes


class KernelProbe:
    """Brackets every launch of the named C-ABI entry points with HIP events on the stream
    the kernel runs on (torch's current stream), to time them live inside the bench."""

    def __init__(self, names, flop_fn):
        self.names = (names,) if isinstance(names, str) else tuple(names)
        self.name = "/".join(self.names)
        self.flop_fn = flop_fn
        self.events = []
        self.flops = []
        self.active = False

    def install(self):
        from ds2amd import _lib
        orig = _lib.call
        probe = self

        def call(name, *args):
            if probe.active and name in probe.names:
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                orig(name, *args)
                e.record()
                probe.events.append((s, e))
                probe.flops.append(probe.flop_fn(args))
            else:
                orig(name, *args)
        _lib.call = call

    def summary(self):
        torch.cuda.synchronize()
        if not self.events:
            return None
        ms = [s.elapsed_time(e) for s, e in self.events]
        return sum(ms) / len(ms), sum(self.flops) / len(self.flops), len(ms)


PMC_SUMMARY = "r9z_pmc_traffic.csv"   # profiles/: PMC passes on the final round-6 tree


def pmc_traffic_per_launch(prefix="gemm", extra=("splitk_reduce_kernel",)):
    """HBM bytes per ds2_sgemm_ws launch from the newest committed PMC summary
    (profiles/r*_pmc_traffic.csv, made by scripts/pmc_traffic.sh + pmc_summary.py:
    FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, one pass per counter)."""
    import csv
    import glob
    # the summary measured on the current kernels; else the last one by name
    cur = os.path.join(REPO, "profiles", PMC_SUMMARY)
    files = ([cur] if os.path.exists(cur) else
             sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_traffic.csv"))))
    if not files:
        return None, None
    launches, total = 0, 0.0
    try:
        rows = list(csv.DictReader(open(files[-1])))
    except (OSError, csv.Error):
        return None, None
    for r in rows:
        name = r.get("kernel", "")
        try:
            calls = int(r["calls"])
        except (KeyError, TypeError, ValueError):
            continue
        if prefix in name and not any(e in name for e in extra):
            launches += calls
            total += calls * float(r["avg_total_MB"])
        elif any(e in name for e in extra):
            total += calls * float(r["avg_total_MB"])
    if launches == 0:
        return None, None
    return total / launches * 1e6, os.path.relpath(files[-1], REPO)


def sgemm_flops(args):
    m, n, k = args[2], args[3], args[4]
    return 2.0 * m * n * k


def gru_recurrence_flops(args):
    """ds2_gru_fwd / ds2_gru_bwd[_bias] (t_max, n, h, num_dirs, ...): the W_hh contraction of
    every step, 2 * T * N * D * 3H * H (backward: the same product with W_hh^T)."""
    t, n, h, d = args[0], args[1], args[2], args[3]
    return 2.0 * t * n * d * 3 * h * h


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cpu_threads() -> int:
    """The host cores this process may use: the box's share (OMP_NUM_THREADS, set to 16 per
    GPU on the pool; os.cpu_count() there counts the whole machine), else the affinity set."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _progress(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(train_steps: int = 3, fwd_steps: int = 2, budget_s: float = 150.0):
    """BASELINE.md §4 / SURVEY §8(d): the oracle (the reference's stock torch CPU op set:
    conv2d / batch_norm / packed nn.GRU / ctc_loss / SGD) on the SAME cfg2 batch the GPU
    trains on (32 x 10 s, 5 x BiGRU-800, seed 123456), all usable host threads, 1 warm-up +
    ``train_steps`` timed training steps, plus a train-mode forward-only figure (1 warm-up +
    ``fwd_steps`` timed).  Medians reported.  Timed training steps stop (never below one) once
    another would exceed ``budget_s``, so the default bench run stays within a few minutes;
    the sample string says what ran."""
    from oracle import ds2_oracle as orc
    from ds2amd import model as dsm
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(123456)
    m = dsm.DeepSpeech(rnn_type='gru', labels=LABELS, rnn_hidden_size=HIDDEN, nb_layers=LAYERS,
                       audio_conf=CONF, bidirectional=True)
    o = orc.OracleDS2({k: v.detach() for k, v in m.state_dict().items()}, LAYERS, HIDDEN)
    x, tg, pct, ts = synthetic_batch(0)
    sizes = orc.input_sizes_quirk(pct, x.shape[3])
    train_t, fwd_t = [], []
    # warm-up: one train step on 2 of the utterances (allocator, thread pool, kernels); a
    # full-batch warm-up step would double the baseline's cost (≈2 min per bs32 step on 16
    # cores: the packed-GRU backward dominates) for a sub-percent effect
    t0 = time.perf_counter()
    orc.train_step(o, x[:2], pct[:2].clone(), tg[:2 * LABEL_LEN], ts[:2])
    _progress(f"cpu baseline: warm-up step (2 utterances) {time.perf_counter() - t0:.1f} s "
              f"on {threads} threads")
    t_start = time.perf_counter()
    for i in range(train_steps):
        t0 = time.perf_counter()
        orc.train_step(o, x, pct.clone(), tg, ts)
        train_t.append(time.perf_counter() - t0)
        _progress(f"cpu baseline: train step {i + 1}/{train_steps} {train_t[-1]:.1f} s")
        if time.perf_counter() - t_start + train_t[-1] > budget_s:
            break
    with torch.no_grad():
        for i in range(1 + fwd_steps):
            t0 = time.perf_counter()
            o.forward(x, sizes, training=True)
            if i > 0:
                fwd_t.append(time.perf_counter() - t0)
            _progress(f"cpu baseline: forward {i}/{fwd_steps} {time.perf_counter() - t0:.1f} s")
    med = lambda v: sorted(v)[len(v) // 2]
    tr, fw = med(train_t), med(fwd_t)
    return {"value": round(BATCH * SECONDS / tr, 4), "unit": "audio-seconds/sec",
            "cores": threads, "kind": "port", "cpu_model": _cpu_model(),
            "forward_only_value": round(BATCH * SECONDS / fw, 4),
            "train_step_s": [round(v, 3) for v in train_t],
            "forward_s": [round(v, 3) for v in fwd_t],
            "sample": f"oracle train step (fwd+CTC+bwd+clip+SGD) on the cfg2 batch, "
                      f"{BATCH} x 10 s, 5xBiGRU-800, torch CPU fp32 on {threads} threads: "
                      f"1 warm-up step on 2 utterances + {len(train_t)} timed full-batch "
                      f"step(s) (at most {train_steps}, {budget_s:.0f} s budget; median "
                      f"{tr:.1f} s); forward-only "
                      f"(train mode, no grad): 1 warm-up + {fwd_steps} timed (median {fw:.1f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3,
                    help="timed oracle training steps of the CPU baseline (after 1 warm-up)")
    ap.add_argument("--probe", default="ds2_sgemm_ws,ds2_sgemm_amax_ws",
                    help="comma-separated C-ABI entry points timed as the GEMM family")
    ap.add_argument("--input", choices=["spect", "pcm"], default="spect",
                    help="spect: 10 s spectrograms resident in HBM (the headline metric); "
                         "pcm: raw 16 kHz PCM resident in HBM, the device STFT + max_frame "
                         "normalisation inside every timed step (SURVEY 8d secondary variant)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DS2_FORCE_DIST=1 under torchrun exercises the RCCL path even at world size 1
    distributed = world > 1 or os.environ.get("DS2_FORCE_DIST") == "1"
    from ds2amd import model as dsm
    from ds2amd.trainer import Trainer, init_distributed
    if distributed:
        init_distributed("nccl", local)            # RCCL over xGMI, channel cap
    dev = torch.device("cuda", local)

    torch.manual_seed(123456)
    m = dsm.DeepSpeech(rnn_type='gru', labels=LABELS, rnn_hidden_size=HIDDEN, nb_layers=LAYERS,
                       audio_conf=CONF, bidirectional=True)
    # score=True: the reference computes CER/WER of the greedy decode every batch
    # (train.py:575-591); here on the device (ds2_edit_distance), inside the timed step
    tr = Trainer(m, LABELS, lr=3e-4, momentum=0.9, max_norm=100.0, device=dev, score=True,
                 verbose=False)
    x, tg, pct, ts = synthetic_batch(rank)
    x = x.to(dev)                                      # inputs resident in HBM
    featurize = None
    if args.input == "pcm":
        from ds2amd import ops
        from ds2amd.data_loader import SpectrogramParser
        parser = SpectrogramParser(CONF, normalize='max_frame', device=dev)
        n_fft, hop, win, taps = parser._consts(16000)
        g = torch.Generator().manual_seed(99 + rank)
        n_samp = int(SECONDS * 16000)
        pcm = torch.rand(BATCH, n_samp, generator=g).mul_(2).sub_(1).to(dev)
        ns = torch.full((BATCH,), n_samp, dtype=torch.int32, device=dev)
        frames = 1 + n_samp // hop

        def featurize():
            return ops.stft_logmag(pcm, ns, n_fft, hop, win, 1, taps, frames).unsqueeze(1)

    probe = KernelProbe(tuple(args.probe.split(",")), sgemm_flops)
    probe.install()
    fprobe = KernelProbe(("ds2_gru_fwd",), gru_recurrence_flops)
    fprobe.install()
    bprobe = KernelProbe(("ds2_gru_bwd", "ds2_gru_bwd_bias", "ds2_gru_bwd_bias_amax"),
                         gru_recurrence_flops)
    bprobe.install()
    aprobe = KernelProbe(("ds2_amax",), lambda a: 4.0 * a[1] * a[2])   # bytes read
    aprobe.install()
    probes = (probe, fprobe, bprobe, aprobe)

    def step():
        inp = x if featurize is None else featurize()
        return tr.train_batch((inp, tg, None, pct.clone(), ts))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    for p_ in probes:
        p_.active = True
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.steps):
        loss = step()
        marks[i + 1].record()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for p_ in probes:
        p_.active = False
    tr.poll_status(block=True)      # raises Ds2Error if a recurrence hand-off failed
    step_ms = sorted(marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps))
    median_ms = step_ms[len(step_ms) // 2]
    if distributed:
        tt = torch.tensor([dt], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    final_loss = float(loss.item())
    pk, fk, bk, ak = (p_.summary() for p_ in probes)

    if rank == 0:
        audio = world * BATCH * SECONDS * args.steps
        value = audio / dt
        ms_per_step = dt * 1000.0 / args.steps
        step_tf = round(TRAIN_FLOP_PER_STEP / (ms_per_step * 1e-3) / 1e12, 3)
        kernels = {}

        def entry(name, summ, peak, arith, bound, pmc):
            if summ is None:
                return
            avg_ms, flop, count = summ
            achieved = flop / (avg_ms * 1e-3) / 1e12
            traffic, src = pmc_traffic_per_launch(*pmc)
            e = {"bound": bound, "kernel": name, "launches": count,
                 "launches_per_step": round(count / args.steps, 2),
                 "avg_launch_ms": round(avg_ms, 5),
                 "ms_per_step": round(avg_ms * count / args.steps, 3),
                 "achieved": round(achieved, 3), "peak": round(peak, 1), "unit": "TFLOP/s",
                 "arith": arith, "frac": round(achieved / peak, 4),
                 # the same work against the dense fp32 MFMA peak (the dtype's own peak; the
                 # bf16x6 kernels run their fp32 products on the bf16 engine, `frac` above)
                 "frac_fp32_mfma_peak": round(achieved / PEAK_F32_MFMA_TFLOPS, 4),
                 "traffic": None if traffic is None else round(traffic),
                 "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": src,
                 "step_achieved_tflops": step_tf}
            if name == "ds2_sgemm_ws" and gemm_mode() in MEASURED_CEILING:
                ceil = MEASURED_CEILING[gemm_mode()]
                e["measured_ceiling"] = ceil
                e["frac_of_measured_ceiling"] = round(achieved / ceil, 4)
                e["ceiling_source"] = CEILING_SOURCE
            if name.startswith("ds2_gru"):
                # latency-bound: T' dependent steps, one cross-CU hand-off each
                e["us_per_step"] = round(avg_ms * 1e3 / ((T_FRAMES - 1) // 2 + 1), 3)
            kernels[name] = e

        gpeak, garith = gemm_peak()
        # the GEMM family: ds2_sgemm_ws and ds2_sgemm_amax_ws (the RNN gradients with shared
        # fp16x3 operand scales), keyed "ds2_sgemm_ws"
        entry("ds2_sgemm_ws", pk, gpeak, garith, "mfma", ("gemm", ("splitk_reduce_kernel",)))
        kernels["ds2_sgemm_ws"]["entry_points"] = args.probe.split(",")
        if ak is not None:
            a_ms, a_bytes, a_n = ak
            kernels["ds2_amax"] = {
                "bound": "hbm", "kernel": "ds2_amax", "launches": a_n,
                "launches_per_step": round(a_n / args.steps, 2),
                "avg_launch_ms": round(a_ms, 5), "ms_per_step": round(a_ms * a_n / args.steps, 3),
                "achieved": round(a_bytes / (a_ms * 1e-3) / 1e9, 1), "unit": "GB/s",
                "peak": 8000.0, "frac": round(a_bytes / (a_ms * 1e-3) / 1e9 / 8000.0, 4),
                "note": "fp16x3 operand row/column maxima shared by the RNN gradient GEMMs "
                        "(one read of each operand)"}
        x6f = _env_on("DS2_GRU_X6")
        fpeak, farith, fkern = gru_fwd_kernel(x6f)
        entry("ds2_gru_fwd", fk, fpeak, farith, "mfma", (fkern, ()))
        bpeak, barith, bkern = gru_bwd_kernel(x6f)
        entry("ds2_gru_bwd", bk, bpeak, barith, "mfma", (bkern, ()))
        # the roofline object is the dominant kernel family of the step (most ms per step)
        roof = max(kernels.values(), key=lambda e: e["ms_per_step"]) if kernels else None
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.cpu_steps)
        out = {
            "metric": "audio-seconds/sec training, DS2 5x BiGRU-800 bs32, at 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "audio-seconds/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "ms_per_step_median": round(median_ms, 3),
            "value_at_median": round(world * BATCH * SECONDS / (median_ms * 1e-3), 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic 10 s spectrograms [32,1,161,1001] + 150-label targets, random init"
                     if featurize is None else
                     "synthetic 10 s 16 kHz PCM [32,160000] -> device STFT + max_frame per step, "
                     "150-label targets, random init"),
            "config": {"workload": "DS2 5x BiGRU-800, 10 s utterances, batch 32 per GPU, "
                                   "CTC training step (cfg2/cfg3)",
                       "global_batch": BATCH * world, "seq_len": T_FRAMES,
                       "parallelism": f"dp{world}"},
            "loss": round(final_loss, 4),
            "dp": {"process_group": distributed, "world": world,
                   "allreduce": "ds2_allreduce_bucket" if tr.reducer.comm is not None
                                else "torch.distributed",
                   "buckets": len(tr.reducer.buckets),
                   "bucket_mb": [round((e - s) * 4 / 2**20, 2) for s, e, _ in tr.reducer.buckets],
                   "issued_from_hooks": tr.reducer.issued_from_hooks,
                   "guard_waits": tr.reducer.guard_waits,
                   "collectives": tr.reducer.collectives,
                   "issue_policy": tr.reducer.policy,
                   "status_in_last_bucket": bool(tr.flat.tail.numel()),
                   "traffic_standin": (None if tr.reducer.standin is None else
                                       {"busbw_gbps": tr.reducer.standin.busbw,
                                        "world": tr.reducer.standin.world,
                                        "ctas": tr.reducer.standin.ctas}),
                   "rccl_cta_cap": tr.reducer.rccl_ctas,
                   "broadcasts": tr.sync.broadcasts,
                   "status_clean": True},
            "roofline": roof,
            "kernels": kernels,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    tr.close()
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    if os.environ.get("DS2_CLEAN_EXIT") == "1":
        # release every device object of the run before the interpreter's exit handlers
        # (exit-time teardown diagnostics, scripts/prof_exit_probe2.sh)
        import gc
        torch.cuda.synchronize()
        del tr, m, x, probe, fprobe, bprobe, aprobe, probes
        gc.collect()
        torch.cuda.empty_cache()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
