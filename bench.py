#!/usr/bin/env python
"""bench.py — single-batch decode throughput of the MI355X path (BASELINE.json metric).

metric: decode tok/s + %HBM-roofline, Mistral-7B fp16, 1x MI355X vs -d cpu.

A "step" is one greedy decode token: argmax over the logits + one full forward pass
(embed -> 32 layers -> final norm -> lm_head), replayed from a hipGraph by the device-side
decode loop (xh_decode_greedy).  Workload (BASELINE configs[1]): Mistral-7B-Instruct-v0.2
shapes, fp16 weights, 4k context, a 32-token prompt (BOS + LCG ids) hydrated first, then
`--warmup` untimed and `--steps` timed decode tokens.  Weights are synthetic (no checkpoints
offline): generated on the device from include/xalm_synth.h; the CPU baseline builds the
bit-identical host copy and runs the C oracle (the reference's CPU algorithm restated).

Multi-GPU: the path does not shard -> N independent replicas, one process per
GPU, no collective on the data path; value = total tokens of all ranks / max rank time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from xalm_amd import _lib as L  # noqa: E402
from xalm_amd.model import InferenceState, Model  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

WORKLOADS = {
    # BASELINE.json configs[1]
    "mistral-7b-f16": dict(desc="Mistral-7B-Instruct-v0.2 fp16, greedy decode, 4k context (configs[1])",
                           dim=4096, hidden=14336, layers=32, heads=32, kv_heads=8, head_dim=128, vocab=32000,
                           msl=4096, theta=1e6, wdt=L.F16, edt=L.F16, cdt=L.F16, dtype="f16", kv_prefill=0),
    # configs[2]: fp8 matrices, embed/lm_head boosted to bf16 (convert.py:729-768)
    "mistral-7b-f8": dict(desc="Mistral-7B fp8 e4m3 weights (embed/lm_head bf16), greedy decode, 4k context (configs[2])",
                          dim=4096, hidden=14336, layers=32, heads=32, kv_heads=8, head_dim=128, vocab=32000,
                          msl=4096, theta=1e6, wdt=L.F8_E4M3, edt=L.BF16, cdt=L.BF16, dtype="f8_e4m3", kv_prefill=0),
    # configs[3]: -T 32768, KV ring pre-filled, decode at pos >= 32767 (KV-dominated)
    "mistral-7b-f16-32k": dict(desc="Mistral-7B fp16, -T 32768, KV ring full (configs[3])",
                               dim=4096, hidden=14336, layers=32, heads=32, kv_heads=8, head_dim=128, vocab=32000,
                               msl=32768, theta=1e6, wdt=L.F16, edt=L.F16, cdt=L.F16, dtype="f16",
                               kv_prefill=32767),
    # configs[4]
    "llama3-8b-f16": dict(desc="Llama-3-8B fp16, greedy decode, 4k context (configs[4])",
                          dim=4096, hidden=14336, layers=32, heads=32, kv_heads=8, head_dim=128, vocab=128256,
                          msl=4096, theta=5e5, wdt=L.F16, edt=L.F16, cdt=L.F16, dtype="f16", kv_prefill=0),
    # SURVEY 8f-4 (not a BASELINE config): the converter's gguf blocks, every matrix including
    # embed / lm_head (convert.py boost_type leaves gguf targets as they are)
    "mistral-7b-q8_0": dict(desc="Mistral-7B gguf Q8_0 blocks (convert.py --type q8_0), greedy decode, 4k context",
                            dim=4096, hidden=14336, layers=32, heads=32, kv_heads=8, head_dim=128, vocab=32000,
                            msl=4096, theta=1e6, wdt=L.Q8_0, edt=L.Q8_0, cdt=L.Q8_0, dtype="q8_0", kv_prefill=0),
    "mistral-7b-q4_0": dict(desc="Mistral-7B gguf Q4_0 blocks (convert.py --type q4_0), greedy decode, 4k context",
                            dim=4096, hidden=14336, layers=32, heads=32, kv_heads=8, head_dim=128, vocab=32000,
                            msl=4096, theta=1e6, wdt=L.Q4_0, edt=L.Q4_0, cdt=L.Q4_0, dtype="q4_0", kv_prefill=0),
}


def make_config(w):
    c = L.XhConfig()
    c.dim, c.hidden_dim, c.head_dim, c.n_layers = w["dim"], w["hidden"], w["head_dim"], w["layers"]
    c.n_heads, c.n_kv_heads, c.vocab_size, c.max_seq_len = w["heads"], w["kv_heads"], w["vocab"], w["msl"]
    c.rope_theta, c.rotary_dim, c.norm_eps, c.act = w["theta"], w["head_dim"], 1e-5, L.ACT_SILU
    c.qkv_clip = float(np.finfo(np.float32).max)
    c.tie_word_embeddings = 0
    return c


def tensor_specs(w, seed_shift=0):
    """(kind, layer, dtype, seed, mean, std) of every tensor; SURVEY §8d synthetic recipe:
    matrices N(0,0.02^2), norms 1+N(0,0.01^2) bf16, embedding rows N(0,1).  seed_shift: another
    draw of the same recipe (a second weight seed for the parity tests)."""
    z = seed_shift
    specs = [(L.EMBED, 0, w["edt"], 1001 + z, 0.0, 1.0), (L.FINAL_NORM, 0, L.BF16, 1002 + z, 1.0, 0.01),
             (L.WCLS, 0, w["cdt"], 1003 + z, 0.0, 0.02)]
    for layer in range(w["layers"]):
        base = 10_000 + 100 * layer + z
        specs += [(L.ATTN_NORM, layer, L.BF16, base + 1, 1.0, 0.01), (L.FFN_NORM, layer, L.BF16, base + 2, 1.0, 0.01)]
        for k in (L.WQ, L.WK, L.WV, L.WO, L.W1, L.W2, L.W3):
            specs.append((k, layer, w["wdt"], base + 10 + k, 0.0, 0.02))
    return specs


def tensor_shape(c, kind):
    q_dim, kv_dim = c.n_heads * c.head_dim, c.n_kv_heads * c.head_dim
    return {L.EMBED: (c.vocab_size, c.dim), L.WCLS: (c.vocab_size, c.dim), L.FINAL_NORM: (1, c.dim),
            L.ATTN_NORM: (1, c.dim), L.FFN_NORM: (1, c.dim), L.WQ: (q_dim, c.dim), L.WK: (kv_dim, c.dim),
            L.WV: (kv_dim, c.dim), L.WO: (c.dim, q_dim), L.W1: (c.hidden_dim, c.dim),
            L.W2: (c.dim, c.hidden_dim), L.W3: (c.hidden_dim, c.dim)}[kind]


def prompt_tokens(vocab, n=32, seed=7):
    out, s = [1], seed
    for _ in range(n - 1):
        s = (1103515245 * s + 12345) & 0x7FFFFFFF
        out.append(3 + s % (vocab - 3))
    return out


def pmc_traffic(kernel_prefix):
    """Read bytes per dispatch of a kernel from the newest committed PMC summary
    (profiles/*_pmc.json, written by tools/pmc.sh: FETCH_SIZE x2 + WRITE_SIZE, separate
    rocprofv3 passes).  None when no summary covers the kernel."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*_pmc.json")))
    for f in reversed(files):
        with open(f) as fh:
            ks = json.load(fh)["kernels"]
        for name, v in ks.items():
            if name.startswith(kernel_prefix) and v.get("read_bytes_avg") is not None:
                return int(v["read_bytes_avg"] + (v.get("write_bytes_avg") or 0)), os.path.basename(f)
    return None, None


def sync_all(dist, torch_mod):
    if torch_mod is not None and torch_mod.cuda.is_available():
        torch_mod.cuda.synchronize()
    if dist is not None:
        dist.barrier()


def timed_region(dist, torch_mod, fn):
    """fn() bracketed by a barrier + device sync on both sides; returns (fn's result, the MAX
    over ranks of the wall time), so every rank reports the slowest replica's time."""
    sync_all(dist, torch_mod)
    t0 = time.perf_counter()
    out = fn()
    sync_all(dist, torch_mod)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    return out, elapsed


def job_value(world, steps, elapsed):
    """whole-job decode throughput: every replica decodes `steps` tokens (weak scaling)"""
    return world * steps / elapsed


def host_cpu_info():
    """lscpu model name, physical cores of the host, and the CPUs this process may run on (the
    GPU box gives one GPU's share of the host: OMP_NUM_THREADS and the affinity mask say how many)."""
    info = {"model": None, "physical_cores": None, "logical_cpus": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        kv = {}
        for line in out.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                kv[k.strip()] = v.strip()
        info["model"] = kv.get("Model name")
        sockets, cores = int(kv.get("Socket(s)", "0") or 0), int(kv.get("Core(s) per socket", "0") or 0)
        info["physical_cores"] = sockets * cores or None
    except Exception:  # lscpu missing: the fields stay null
        pass
    return info


def usable_physical_cores():
    """Physical cores (distinct package / core ids) among the CPUs in this process's affinity
    mask, capped by a cgroup CPU quota if one is set: the cores a `-d cpu` run here can use
    (BASELINE.md §3 asks for OMP_NUM_THREADS = all physical cores)."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    phys = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                pkg = f.read().strip()
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                core = f.read().strip()
            phys.add((pkg, core))
        except OSError:
            phys.add(("cpu", c))
    n, quota = len(phys), None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
            n = min(n, max(1, int(quota)))
    except (OSError, ValueError):
        pass
    return max(1, n), quota


def progress(msg):
    """A progress line on stderr (the JSON result is the only stdout line)."""
    print(msg, file=sys.stderr, flush=True)


def cpu_baseline(w, c, prompt, gpu_logits0, gpu_tokens, n_decode, one_thread_tokens=2, share_tokens=8):
    """The reference -d cpu path (the oracle: src/infer.cpp restated, OpenMP over matvec rows and
    heads as src/infer.cpp:118 / :438) on the same synthetic weights, timed on this host with
    OpenMP threads = the physical cores this process may use: hydrate the prompt,
    then `n_decode` decode tokens teacher-forced on the GPU's tokens (run_completion -m completion
    -n N, src/main.cpp:94-115), as wall tok/s and as the reference's own statistic (prompt +
    generated) / (user + sys CPU s) (src/main.cpp:117-127, src/profiler.h:124-129; NOT wall
    clock).  Beside it: the same decode at the GPU box's CPU share (OMP_NUM_THREADS as set for the
    job) and on one thread.  Parity of the same run: GPU logits after the prompt against the
    oracle's f32 evaluation and against the fp64 evaluation of the same algorithm
    (xo_set_precision), with the f32 evaluation's own distance from the fp64 one."""
    import resource

    from oracle import oracle as O
    t_gen = time.time()
    weights = [(kind, layer, dt, O.synthetic(*tensor_shape(c, kind), dt, seed, mean, std))
               for kind, layer, dt, seed, mean, std in tensor_specs(w)]
    kv_rows = []
    pos0, hyd = 0, prompt
    if w["kv_prefill"]:
        kv_dim = c.n_kv_heads * c.head_dim
        for layer in range(c.n_layers):
            if layer % 8 == 0:
                progress(f"cpu baseline: KV history layer {layer} / {c.n_layers}")
            for which in (0, 1):
                kv_rows.append((layer, which, O.synthetic(w["kv_prefill"], kv_dim, L.F16, 5000 + 2 * layer + which,
                                                          0.0, 1.0)))
        pos0, hyd = w["kv_prefill"], prompt[:1]

    def oracle(prec=0):
        om = O.OracleModel(c)
        for kind, layer, dt, arr in weights:
            om.set_tensor(kind, layer, dt, arr)
        for layer, which, arr in kv_rows:
            om.set_kv(layer, which, 0, arr)
        om.set_precision(prec)
        return om

    om = oracle()
    t_gen = time.time() - t_gen
    progress(f"cpu baseline: weights ready ({t_gen:.1f} s)")
    share = O.num_threads()  # the job's OMP_NUM_THREADS (the GPU box's CPU share)
    cores, quota = usable_physical_cores()
    O.set_threads(cores)
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.time()
    for i, tok in enumerate(hyd):
        if i % 8 == 0:
            progress(f"cpu baseline: hydrate token {i} / {len(hyd)}")
        om.forward(tok, pos0 + i, L.OUTPUT_LOGITS if i == len(hyd) - 1 else L.HYDRATE_KV_CACHE)
    t_hyd = time.time() - t0
    lg0 = om.logits()
    # teacher-forced on the GPU's tokens so both sides see identical inputs
    pos = pos0 + len(hyd)
    # bytes the decode tokens move (Model::active_bytes, src/model.cpp:12-35): the CPU's GB/s
    dec_bytes = sum(om.active_bytes(pos + i) for i in range(n_decode))
    agree, disagree = 0, []
    t1 = time.time()
    for i in range(n_decode):
        if i % 16 == 0 or w["kv_prefill"]:
            progress(f"cpu baseline: decode token {i} / {n_decode} ({cores} threads)")
        lg = om.logits()
        ref_tok = O.sample_argmax(lg)
        if ref_tok == gpu_tokens[i]:
            agree += 1
        else:  # the logit gap the two paths saw at this step (a near-tie if below the error)
            disagree.append({"step": i, "gpu": int(gpu_tokens[i]), "oracle": int(ref_tok),
                             "oracle_logit_gap": float(lg[ref_tok] - lg[gpu_tokens[i]])})
        om.forward(gpu_tokens[i], pos, L.OUTPUT_LOGITS)
        pos += 1
    t_dec = time.time() - t1
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)

    nxt = n_decode  # the next teacher-forcing token

    def sample(threads, n_tok):
        nonlocal pos, nxt
        O.set_threads(threads)
        t = time.time()
        for k in range(n_tok):
            progress(f"cpu baseline: {threads}-thread sample, token {k} / {n_tok}")
            om.forward(gpu_tokens[nxt], pos, L.OUTPUT_LOGITS)
            pos += 1
            nxt += 1
        return n_tok / (time.time() - t)

    # the job's CPU share and one thread, a few more teacher-forced tokens each
    share_tps = sample(share, share_tokens) if share != cores else n_decode / t_dec
    one_tps = sample(1, one_thread_tokens)
    O.set_threads(cores)
    om.close()
    # fp64 evaluation of the same prompt (the algorithm's value independent of f32 rounding order)
    t2 = time.time()
    om64 = oracle(1)
    for i, tok in enumerate(hyd):
        if i % 4 == 0:
            progress(f"cpu baseline: fp64 evaluation, token {i} / {len(hyd)}")
        om64.forward(tok, pos0 + i, L.OUTPUT_LOGITS if i == len(hyd) - 1 else L.HYDRATE_KV_CACHE)
    lg64 = om64.logits()
    om64.close()
    t_64 = time.time() - t2
    O.set_threads(share)
    cpu = host_cpu_info()
    return dict(value=round(n_decode / t_dec, 3), unit="tok/s", cores=cores, kind="port",
                achieved_GBps=round(dec_bytes / t_dec / 1e9, 1),
                isa={2: "AVX-512 (run-time dispatch)", 1: "AVX2/FMA/F16C", 0: "scalar"}[O.isa()],
                cpu_model=cpu["model"], host_physical_cores=cpu["physical_cores"],
                host_logical_cpus=cpu["logical_cpus"], affinity_cpus=cpu["affinity_cpus"], cgroup_cpu_quota=quota,
                threads_note="OpenMP threads = the physical cores in this process's affinity mask (capped by a "
                             "cgroup quota if set), BASELINE.md §3",
                sample=f"-m completion -n {n_decode} equivalent: {len(hyd)}-token hydrate"
                       + (f" at pos {pos0} over a {w['kv_prefill']}-slot history" if w["kv_prefill"] else "")
                       + f", then {n_decode} greedy decode tokens teacher-forced on the GPU's tokens, full "
                       f"{w['desc'].split(',')[0]} shapes, same synthetic weights (wall clock, OpenMP "
                       "oracle/xalm_oracle.c = the reference's CPU algorithm restated)",
                ms_per_token=round(1000 * t_dec / n_decode, 2),
                hydrate_s=round(t_hyd, 3), weight_gen_s=round(t_gen, 2),
                reference_stat={"value": round((len(hyd) + n_decode) / cpu_s, 3) if cpu_s > 0 else None,
                                "unit": "tok/s", "definition": "(prompt + generated) / (user + sys CPU s), "
                                "src/main.cpp:117-127 + src/profiler.h:124-129; NOT wall clock",
                                "user_sys_s": round(cpu_s, 2)},
                job_share={"value": round(share_tps, 3), "unit": "tok/s", "cores": share,
                           "sample": f"{share_tokens if share != cores else n_decode} teacher-forced decode tokens at "
                                     "the job's OMP_NUM_THREADS"},
                one_thread={"value": round(one_tps, 3), "unit": "tok/s", "cores": 1,
                            "sample": f"{one_thread_tokens} teacher-forced decode tokens"},
                parity={"gpu_vs_oracle32_max_abs": float(np.abs(lg0 - gpu_logits0).max()),
                        "gpu_vs_oracle64_max_abs": float(np.abs(lg64 - gpu_logits0).max()),
                        "oracle32_vs_oracle64_max_abs": float(np.abs(lg64 - lg0).max()),
                        "logits_scale": float(np.abs(lg64).max()),
                        "note": "logits after the prompt; oracle64 = the same algorithm evaluated in double "
                                "(fp16 K/V cache kept); the GPU passes when it is no further from oracle64 than "
                                "the reference's own f32 evaluation (tests/test_parity_full_gpu.py)",
                        "oracle64_s": round(t_64, 1),
                        "greedy_tokens_agree": f"{agree}/{n_decode}", "disagreements": disagree[:16]})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--workload", default="mistral-7b-f16", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-tokens", type=int, default=128,
                    help="CPU baseline decode tokens (-m completion -n N; 32k workload: min(N, 32))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=200)
    ap.add_argument("--prefill-mode", type=int, default=1, choices=(1, 2, 3, 4),
                    help="batched prefill GEMMs (XH_OPT_PREFILL): 1 default per dtype (the LDS-tiled f16 MFMA "
                         "GEMM of gemm16.h for f16 / fp8 weights), 2 split-f16 register-streaming MFMA wherever "
                         "the weights allow, 3 f32-input MFMA only, 4 as 1 on vendor hipBLASLt")
    ap.add_argument("--prefill-tokens", type=int, default=2048,
                    help="also time xh_prefill of this many prompt tokens (batched path; 0 = skip)")
    ap.add_argument("--fuse-attn-wo", type=int, default=1, choices=(0, 1),
                    help="attention + Wo in one launch (1) or two launches (0)")
    ap.add_argument("--pos0", type=int, default=0,
                    help="4k workloads: ring slots [0, pos0) hold a synthetic K/V history and the prompt is "
                         "hydrated at pos0 (e.g. 3808: the timed tokens end at kv_len 4096, the worst token of "
                         "the 4k context, SURVEY 8d)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    torch_mod = None
    try:
        import torch as torch_mod  # noqa: F811  (plumbing: barrier + device sync only)
    except ImportError:
        torch_mod = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)

    w = WORKLOADS[args.workload]
    c = make_config(w)
    # XALM_BENCH_DEVICE: every rank on one device (a multi-rank rehearsal on a one-GPU box)
    device = int(os.environ.get("XALM_BENCH_DEVICE", local_rank))
    model = Model(c, device=device)
    for kind, layer, dt, seed, mean, std in tensor_specs(w):
        model.upload_synthetic(kind, layer, dt, seed, mean, std)

    model.set_option(L.OPT_FUSE_ATTN_WO, args.fuse_attn_wo)
    prompt = prompt_tokens(c.vocab_size)
    st = InferenceState(c)
    pos0 = 0
    if w["kv_prefill"]:
        # configs[3]: ring slots 0..kv_prefill-1 hold history; decode continues at pos = kv_prefill
        for layer in range(c.n_layers):
            model.kv_fill_synthetic(layer, 0, 0, w["kv_prefill"], 5000 + 2 * layer, 1.0)
            model.kv_fill_synthetic(layer, 1, 0, w["kv_prefill"], 5001 + 2 * layer, 1.0)
        pos0 = w["kv_prefill"]
    elif args.pos0:
        if args.pos0 + len(prompt) + args.warmup + args.steps > c.max_seq_len:
            raise SystemExit(f"--pos0 {args.pos0}: prompt + warmup + steps exceed the {c.max_seq_len} context")
        for layer in range(c.n_layers):
            model.kv_fill_synthetic(layer, 0, 0, args.pos0, 5000 + 2 * layer, 1.0)
            model.kv_fill_synthetic(layer, 1, 0, args.pos0, 5001 + 2 * layer, 1.0)
        pos0 = args.pos0
    model.prefill(prompt[:1] if w["kv_prefill"] else prompt, pos0, st)
    pos = pos0 + (1 if w["kv_prefill"] else len(prompt))
    logits0 = st.logits().copy()
    if args.pos0 and not w["kv_prefill"]:
        args.no_cpu_baseline = True  # the CPU baseline's oracle starts from an empty ring

    warm_tokens = model.decode_greedy(pos, args.warmup) if args.warmup else []
    pos += args.warmup
    if pos + args.steps > c.max_seq_len and not w["kv_prefill"]:
        raise SystemExit(f"steps exceed the {c.max_seq_len} context")

    toks, elapsed = timed_region(dist, torch_mod, lambda: model.decode_greedy(pos, args.steps))
    assert len(toks) == args.steps
    # the CPU baseline's teacher-forcing tokens beyond the timed ones (-n 128 whatever --steps is):
    # the same greedy sequence continued on the device, untimed
    cpu_n = 0
    extra = []
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_n = min(args.cpu_tokens, 32) if w["kv_prefill"] else args.cpu_tokens
        need = cpu_n + 2 + 8 - (args.warmup + args.steps)
        if need > 0 and (w["kv_prefill"] or pos + args.steps + need <= c.max_seq_len):
            extra = model.decode_greedy(pos + args.steps, need)

    # algorithmic bytes of the timed tokens: Model::active_bytes(pos) (src/model.cpp:12-35)
    step_bytes = sum(model.active_bytes(p) for p in range(pos, pos + args.steps))
    step_gbps = step_bytes / elapsed / 1e9

    # graph engine's kernels, each timed on its own (HIP events on the context stream)
    kv_len_now = min(c.max_seq_len, pos + args.steps)
    k_us = model.time_kernel(0, args.kernel_iters)
    k_bytes = model.kernel_bytes(0, kv_len_now)
    k_gbps = k_bytes / (k_us * 1e-6) / 1e9
    extra_kernels = {"gemv_w13": {"avg_us": round(k_us, 2), "GBps": round(k_gbps, 1)}}
    timed = [(1, "gemv_qkv"), (2, "gemv_wo"), (3, "gemv_w2"), (4, "gemv_lm_head"), (5, "attention")]
    for which, name in timed:
        us = model.time_kernel(which, max(20, args.kernel_iters // 4))
        b = model.kernel_bytes(which, kv_len_now)
        extra_kernels[name] = {"avg_us": round(us, 2), "GBps": round(b / (us * 1e-6) / 1e9, 1)}

    # prompt processing, reported beside the decode metric: xh_prefill of a
    # synthetic prompt at positions 0.. (overwrites the ring rows the decode used; timed last)
    prefill = None
    if args.prefill_tokens and not w["kv_prefill"] and args.prefill_tokens <= c.max_seq_len:
        ptoks = prompt_tokens(c.vocab_size, n=args.prefill_tokens, seed=11)
        model.set_option(L.OPT_PREFILL, args.prefill_mode)
        model.prefill(ptoks, 0, st)  # warm: buffers, code objects, hipBLASLt plans
        sync_all(None, torch_mod)
        t0 = time.perf_counter()
        model.prefill(ptoks, 0, st)
        sync_all(None, torch_mod)
        pf_s = time.perf_counter() - t0
        q_dim, kv_dim = c.n_heads * c.head_dim, c.n_kv_heads * c.head_dim
        layer_params = c.dim * (q_dim + 2 * kv_dim) + q_dim * c.dim + 3 * c.dim * c.hidden_dim
        flops = 2.0 * args.prefill_tokens * c.n_layers * layer_params  # matrix products only
        prefill = {"tokens": args.prefill_tokens, "ms": round(pf_s * 1e3, 2),
                   "tok_s": round(args.prefill_tokens / pf_s, 1),
                   "mode": {0: "per-token", 1: "batched: gemm16.h LDS-tiled f16 MFMA GEMM (f16 / fp8 / gguf-block "
                                               "weights), else register-streaming MFMA kernels",
                            2: "batched split-f16 register-streaming MFMA", 3: "batched f32-input MFMA",
                            4: "batched: hipBLASLt f16 GEMMs (f16 / fp8 weights)"}[model.get_option(L.OPT_PREFILL)],
                   "note": "f16 / fp8 / gguf-block weights: passes of up to 2048 tokens (hipBLASLt: 512), f16 GEMMs "
                           "(fp8 matrices through their exact f16 image, gguf blocks through exact f16 hi + lo images) "
                           "over f16 hi+lo activation pairs (power-of-two row scale, ~22-bit mantissa), hi and lo "
                           "accumulated in f32; other dtypes (bf16, f32, Q8): passes of 64 tokens on the f32-input "
                           "MFMA GEMM (f32 activations as the reference)",
                   "matmul_tflops": round(flops / pf_s / 1e12, 1)}
        # run_perplexity's loop (xh_perplexity): the same tokens, every token's logits and
        # sample_prob of the next one on the device
        t0 = time.perf_counter()
        probs = model.token_probs(ptoks, 0)
        sync_all(None, torch_mod)
        pp_s = time.perf_counter() - t0
        prefill["perplexity"] = {"tokens": len(ptoks) - 1, "ms": round(pp_s * 1e3, 2),
                                 "tok_s": round((len(ptoks) - 1) / pp_s, 1),
                                 "finite": bool(np.isfinite(np.log(probs)).all())}

    # configs[3]: a prompt pass over a long history (the MFMA prompt attention walks slots
    # [0, pos] per workgroup (1) or per wave (2); XH_OPT_PREFILL_ATTN 0 = the split-KV per-token
    # attention), timed at the
    # end of the 32k ring
    if args.prefill_tokens and w["kv_prefill"] and args.prefill_tokens < c.max_seq_len:
        ptoks = prompt_tokens(c.vocab_size, n=args.prefill_tokens, seed=11)
        p0 = c.max_seq_len - args.prefill_tokens - 1
        model.set_option(L.OPT_PREFILL, args.prefill_mode)
        res = {}
        for attn, name in ((1, "mfma_shared_tiles"), (2, "mfma_per_wave_tiles"), (0, "split_kv")):
            model.set_option(L.OPT_PREFILL_ATTN, attn)
            model.prefill(ptoks, p0, st)  # warm
            sync_all(None, torch_mod)
            t0 = time.perf_counter()
            model.prefill(ptoks, p0, st)
            sync_all(None, torch_mod)
            res[name] = round(args.prefill_tokens / (time.perf_counter() - t0), 1)
        model.set_option(L.OPT_PREFILL_ATTN, 1)
        # short passes at the end of the ring (resuming a long chat): the prompt attention's
        # history splits (XH_OPT_PREFILL_ATTN_SPLIT 1) against one walk per workgroup (0)
        short = {}
        for n in (1, 32, 256):
            stoks = prompt_tokens(c.vocab_size, n=n, seed=17)
            p0s = c.max_seq_len - n
            for split in (1, 0):
                model.set_option(L.OPT_PREFILL_ATTN_SPLIT, split)
                model.prefill(stoks, p0s, st)  # warm
                sync_all(None, torch_mod)
                t0 = time.perf_counter()
                model.prefill(stoks, p0s, st)
                sync_all(None, torch_mod)
                short[f"{n}_tok_split{split}_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
        model.set_option(L.OPT_PREFILL_ATTN_SPLIT, 1)
        prefill = {"tokens": args.prefill_tokens, "pos0": p0, "tok_s_by_attention": res,
                   "short_passes_at_ring_end": short,
                   "note": "prompt pass at the end of the -T 32768 ring: each token attends over ~30k slots; "
                           "short_passes: wall ms of one xh_prefill of n tokens at pos0 = 32768 - n"}

    cpu = None
    if cpu_n:
        seq = list(warm_tokens) + list(toks) + list(extra)  # the GPU's greedy tokens after the prompt
        n = min(cpu_n, len(seq) - 2 - 8)  # + 2 one-thread tokens + 8 at the job's thread count
        if n > 0:
            cpu = cpu_baseline(w, c, prompt, logits0, seq, n)

    # the W1/W3 launch's instantiation (the pipelined PF shape, PIPE = 2; the name's prefix, so
    # the trailing GemvShape parameters added since round 6 still match)
    traffic, src = pmc_traffic("void xalm::gemv_kernel<%d, 1, 3, xalm::GemvShape<512, 2, %d, true, 4, true, 2, 2"
                               % (w["wdt"], 2 if w["wdt"] == L.Q4_0 else 4))
    roofline = {"bound": "hbm", "achieved": round(k_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(k_gbps / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "traffic_source": src,
                "kernel": "gemv_kernel<PRO_RMSNORM,EPI_GLU> (fused W1/W3 + rmsnorm + silu*up), layers rotating",
                "bytes_per_launch": k_bytes, "avg_launch_us": round(k_us, 2)}
    value = job_value(world, args.steps, elapsed)
    if rank == 0:
        out = {
            "metric": "decode tok/s + %HBM-roofline, Mistral-7B fp16, 1xMI355X vs -d cpu",
            "value": round(value, 2),
            "unit": "tok/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": w["dtype"],
            "data": "synthetic (deterministic xalm_synth weights of the named shapes; no checkpoint offline)",
            "config": {"workload": w["desc"], "prompt_tokens": len(prompt), "max_seq_len": c.max_seq_len,
                       "history_pos0": pos0,
                       "kv_len_timed": [pos + 1, pos + args.steps], "batch": 1, "parallelism": f"replicas x{world}",
                       "engine": {1: "hipGraph per token, attention+Wo fused",
                                  0: "hipGraph per token"}[model.get_option(L.OPT_FUSE_ATTN_WO)]},
            "roofline": roofline,
            "hbm_step": {"achieved_GBps": round(step_gbps, 1), "frac": round(step_gbps / HBM_PEAK_GBPS, 4),
                         "bytes_per_token": step_bytes // args.steps,
                         "note": "Model::active_bytes per token x tok/s, whole forward incl. launch gaps"},
            "kernels": extra_kernels,
            "cpu_baseline": cpu,
            "prefill": prefill,
        }
        print(json.dumps(out), flush=True)
    model.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
