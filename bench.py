#!/usr/bin/env python
"""Benchmark of the MI355X SketchML gradient codec (BASELINE.json metric).

One step = encode one 2^28-float (1 GiB) fp32 gradient resident in HBM (k=128 quantile sketch ->
getQuantiles(256) -> Maths.unique -> bucket quantise -> packed codes): the north-star
configuration of BASELINE.json ("device-resident encode of a 256 M-float gradient at 1 GPU").
BASELINE config 2 (a 2^26-float bucket) is timed under extras.other_configs.dense_c2.
With --gpus N > 1 every rank encodes its own 2^28-float gradient (weak scaling) and the step adds
the RCCL all-gather of the compressed payloads over xGMI.  `value` = fp32-input GB/s of the whole job.

Extra fields: decode GB/s and decode L2 error (the metric's "+ decode L2 err"), per-kernel
device times, the roofline of the dominant kernel, the CPU baseline (the C restatement of the
reference Java algorithm, oracle/, timed on this host on a bounded sample) and the
H2D/D2H-inclusive rate.
"""
import argparse
import ctypes as C
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md "Chip-level parameters"
KNAMES = {0: "k_leaf", 1: "k_merge", 2: "k_summary", 3: "k_quantize", 4: "k_decode", 5: "k_decode_sum"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warmup-ms", type=float, default=60.0,
                    help="continue the warm-up until this much wall time has passed (the engine clock "
                         "settles after ~25 ms of sustained encodes)")
    ap.add_argument("--n", type=int, default=2**28, help="floats per GPU bucket (default: the north-star 2^28)")
    ap.add_argument("--bins", type=int, default=256)
    ap.add_argument("--buffers", type=int, default=0,
                    help="rotating input buckets so a step never re-reads the previous step's "
                         "input from the 256 MB Infinity Cache (default: 2 of 1 GiB and more, else "
                         "enough for 1 GiB in total)")
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32",
                    help="input dtype (f64 = the reference's double[] path)")
    ap.add_argument("--quant", choices=["quantile", "uniform"], default="quantile")
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="CPU baseline budget (both legs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip decode / H2D measurements")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the fp64 and C3 sparse measurements reported under extras.other_configs")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo group and reports itself")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` without a launcher: start N fresh worker processes of this script,
    one per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them),
    before this process makes any GPU call; forward rank 0's JSON line; fail if any rank fails."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    import threading
    import time as _t
    out0 = []
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    # a rank that dies leaves the others waiting in a collective: stop them (our own children)
    first_bad = []
    while any(p.poll() is None for p in procs):
        first_bad = [r for r, p in enumerate(procs) if p.poll() not in (None, 0)]
        if first_bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        _t.sleep(0.2)
    reader.join(timeout=30)
    rcs = [p.wait() for p in procs]
    bad = first_bad or [r for r, rc in enumerate(rcs) if rc != 0]
    if bad:
        print(f"bench.py: rank(s) {bad} failed with exit codes {[rcs[r] for r in bad]}; all exit codes {rcs}",
              file=sys.stderr)
        return 1
    sys.stdout.write((out0[0] if out0 else b"").decode())
    sys.stdout.flush()
    return 0


def dry_run(args, world: int, rank: int) -> None:
    """Launcher rehearsal on the CPU: gloo group, one all-gather of the ranks, rank 0 reports.
    SKML_DRYRUN_FAIL_RANK=r makes rank r exit with status 3 (the launcher's failure path)."""
    if os.environ.get("SKML_DRYRUN_FAIL_RANK") == str(rank):
        sys.exit(3)
    dist.init_process_group("gloo")
    t = torch.tensor([rank], dtype=torch.int64)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "n_gpus": world, "ranks_seen": [int(v.item()) for v in out],
                          "gpus_arg": args.gpus}))
    dist.destroy_process_group()


def kernel_stats(lib, ctx):
    out = {}
    for kid, name in KNAMES.items():
        n = C.c_int64()
        ms = C.c_double()
        lib.skml_ctx_kernel_stats(ctx, kid, C.byref(n), C.byref(ms))
        if n.value:
            out[name] = {"launches": n.value, "avg_us": 1000.0 * ms.value / n.value}
    return out


def pmc_traffic(kernel, n, dtype="f32", quant="quantile"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary, if one exists
    for this problem size, input type and quantizer (profiles/*pmc*.json, written by
    tools/pmc_summary.py; summaries without dtype/quant keys are fp32 quantile runs)."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        k = d.get("kernels", {}).get(kernel)
        if (k and d.get("n") == n and d.get("dtype", "f32") == dtype and d.get("quant", "quantile") == quant
                and "hbm_bytes_per_launch" in k):
            best = (k["hbm_bytes_per_launch"], os.path.relpath(path, ROOT))
    return best


# VALU issue ceiling of the leaf (wave-instructions / s, whole chip).  tools/ubench/issue.hip on
# gfx950 (profiles/r06_ubench_issue.txt, 8 waves per SIMD of independent chains): v_min/v_max/
# v_med3/v_min3 (f32 and u32), every DPP move or DPP-fused op, v_cmp/v_cndmask_e64, v_bfi/v_perm
# take ~4.4 SIMD cycles per wave-instruction (the 4-cycle rate: one wave-instruction per clock per
# CU), while v_add/v_sub/v_and/v_xor/v_lshr/v_mul_f32/v_fma_f32 take ~2.6 (the SIMD-32 rate, 2
# cycles).  The leaf's code is 7.8 % 2-cycle instructions (tools/valu_mix.py ->
# profiles/r06_leaf_valu_mix.json), so its ceiling is the 4-cycle rate x 4 / (4 - 2 x 0.078) at the
# 2.4 GHz peak engine clock on 256 CUs.
VALU_CLASS_PEAK_GINST = 2.4e9 * 256 / 1e9


def _valu_mix_factor():
    try:
        with open(os.path.join(ROOT, "profiles", "r06_leaf_valu_mix.json")) as f:
            d = json.load(f)
        return float(d["ceiling_factor"]), "profiles/r06_leaf_valu_mix.json"
    except Exception:
        return 1.0, None


VALU_MIX_FACTOR, VALU_MIX_SOURCE = _valu_mix_factor()
VALU_PEAK_GINST = VALU_CLASS_PEAK_GINST * VALU_MIX_FACTOR


def sq_valu(kernel, n):
    """VALU wave-instructions per launch of `kernel` at problem size n from the committed SQ counter
    pass (profiles/*sq_counters.json, written by tools/prof_round.sh; files without an "n" key are
    the 2^26 runs of rounds 1-3)."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*sq_counters.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        if d.get("n", 2**26) != n:
            continue
        for name, c in d.get("per_launch_mean", {}).items():
            short = "k_leaf" if ("k_leaf2" in name or "k_leaf64" in name) else name.split("(")[0].split("::")[-1]
            if short == kernel and "SQ_INSTS_VALU" in c:
                best = (c["SQ_INSTS_VALU"], os.path.relpath(path, ROOT))
    return best


def _affinity():
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def _cpu_threads():
    """Host threads this process may use: the affinity mask, capped by OMP_NUM_THREADS (16 on the
    GPU box, which shares a many-core host)."""
    try:
        t = len(os.sched_getaffinity(0))
    except Exception:
        t = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        t = min(t, int(omp))
    return max(1, t)


def cpu_baseline(x_host, bins, budget_s):
    """The reference's dense encode on this host's cores (oracle/cpu_baseline.cpp, checked against
    the oracle in tests/test_cpu_baseline.py), on bounded samples of the same workload:
      1 thread : QuantileQuantizer.quantize + quantizeToBins (the path ml uses,
                 SketchGradient.scala:27), on the first 2^22 floats of the bucket;
      T threads: parallelQuantize + parallelQuantizeToBins (QuantileQuantizer.java:53-92,
                 Quantizer.java:94-117), T = the usable host threads, on the first 2^24 floats.
    `value` is the faster (threaded) leg."""
    from oracle import oracle as O
    legs = {}
    for name, threads, n in (("1_thread", 1, 2**22), ("threads", _cpu_threads(), 2**24)):
        sample = np.ascontiguousarray(x_host[:n])
        t1 = O.cpu_bench(sample, bins, 1, threads, 1)
        reps = max(1, int(budget_s / 2 / max(t1, 1e-3)))
        t = O.cpu_bench(sample, bins, 1, threads, reps)
        legs[name] = {"gbps": round(4.0 * len(sample) * reps / t / 1e9, 4), "threads": threads,
                      "sample": f"first {len(sample)} floats of the bucket, {reps} encode(s), {t:.1f} s"}
    best = legs["threads"]
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"value": best["gbps"], "unit": "GB/s", "cores": best["threads"], "kind": "port",
            "cores_note": f"{best['threads']} threads: this process's CPU affinity ({_affinity()} CPUs) capped by "
                          f"OMP_NUM_THREADS={omp} (the GPU box's per-job CPU share); the host has {os.cpu_count()}",
            "sample": best["sample"] + " (parallelQuantize + parallelQuantizeToBins)",
            "legs": legs, "cpu": _cpu_model(),
            "what": "oracle/cpu_baseline.cpp: C++ -O3 restatement of the reference Java encode "
                    "(std::sort per 256-value base buffer, sketch merges, getQuantiles, binary-search "
                    "indexOf, 1-byte code write), not a JVM"}


def other_configs(sk, lib, ctx, dev):
    """The reference's other dense / sparse configurations at one GPU, each timed over a few
    synchronised repetitions (not part of `value`): C2 (a 2^26-float bucket), the fp64 path on the
    C2 bucket (the reference's double[] itself), 8 buckets per call, C4's decode-sum and the C3
    sparse path (2^28-dim dense, 10 % nnz) with its aggregation."""
    out = {}
    gen = torch.Generator(device=dev)
    xs = []
    for b in range(4):  # C2: 4 rotating 2^26-float buckets (1 GiB in total, beyond the 256 MB MALL)
        gen.manual_seed(4 + 1000 * b)
        xs.append(torch.randn(2**26, device=dev, generator=gen))
    out["dense_c2"] = dense_bucket(sk, lib, ctx, dev, xs, "C2: 2^26-float dense gradient bucket, 256 requested bins, "
                                   "encode (4 rotating buckets)")
    out["dense_c2"]["parity_test"] = "tests/test_gpu_configs.py::test_c2_full_size_matches_oracle"

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps, r

    def timed_median(fn, reps):
        # median of synchronised repetitions, for the multi-ms sparse calls: one r01h run saw a
        # single stalled C3 rep lift a 3-rep mean from 3.7 ms to 96 ms
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts), r

    n = xs[0].numel()
    gen.manual_seed(4)
    x64 = torch.randn(n, dtype=torch.float64, device=dev, generator=gen)
    nb = lib.skml_dense_payload_bytes(n, 256)
    pl = sk.alloc_aligned(nb, dev)
    p = _lib_params(256)
    t64, _ = timed(lambda: lib.skml_dense_encode_f64(ctx, C.c_void_p(x64.data_ptr()), n, C.byref(p),
                                                      C.c_void_p(pl.data_ptr()), nb), 20)
    out["fp64_encode"] = {"workload": "C2 shape in fp64: 2^26 N(0,1) doubles (generator seed 4), 256 bins",
                          "ms": round(t64 * 1e3, 4), "gbps_fp64_in": round(8.0 * n / t64 / 1e9, 1),
                          "parity_test": "tests/test_gpu_f64_uniform.py::test_f64_bench_workload_2p26_matches_oracle"}
    del x64, pl
    # several independent buckets per call (skml_dense_encode_batch_f32: two streams, so one
    # bucket's VALU-bound sketch overlaps the previous bucket's HBM-bound quantize)
    nbk = 8
    pls = [sk.alloc_aligned(nb, dev) for _ in range(nbk)]
    ptrs = (C.c_void_p * nbk)(*[xs[i % len(xs)].data_ptr() for i in range(nbk)])
    pptr = (C.c_void_p * nbk)(*[q.data_ptr() for q in pls])
    ns = (C.c_int64 * nbk)(*([n] * nbk))
    caps = (C.c_size_t * nbk)(*([nb] * nbk))
    tb, _ = timed(lambda: lib.skml_dense_encode_batch_f32(ctx, nbk, ptrs, ns, C.byref(p), pptr, caps), 10)
    out["batched_buckets"] = {"workload": f"{nbk} independent 2^26-float buckets per call, 256 bins",
                              "ms_per_bucket": round(tb / nbk * 1e3, 4), "gbps": round(4.0 * n * nbk / tb / 1e9, 1),
                              "parity_test": "tests/test_gpu_dense.py::test_quantize_buckets_matches_single_encodes, "
                                             "tests/test_gpu_configs.py::test_c4_consumer_decode_sum_8x2p26_matches_oracle "
                                             "(8 x 2^26 through the batched encode)"}
    del pls, xs
    # the consumers: C4's 8 gathered 2^26-float buckets (bucket r drawn with seed 4 + r, 8-bit codes)
    # and C5's 8 gathered 2^27-float shards (seed 5 + r, 4 requested bins = 2-bit codes)
    out["dense_decode_sum_c4"] = dense_decode_sum(sk, lib, ctx, dev, 2**26, 256, 4)
    out["dense_decode_sum_c4"]["parity_test"] = \
        "tests/test_gpu_configs.py::test_c4_consumer_decode_sum_8x2p26_matches_oracle"
    out["dense_decode_sum_c5"] = dense_decode_sum(sk, lib, ctx, dev, 2**27, 4, 5)
    out["dense_decode_sum_c5"]["parity_test"] = \
        "tests/test_gpu_configs.py::test_c5_consumer_decode_sum_8x2p27_matches_oracle"
    dim = 2**28
    d = c3_dense(dev, 3, dim)
    te, spl = timed_median(lambda: sk.encode_dense_as_sparse(d, 256, 8, 2, 0.3, 3, 3), 5)
    td, (rk, rv) = timed_median(lambda: spl.restore(), 5)
    nnz = int(rk.numel())
    alg = (4.0 + nnz / dim * (8 + 4 + 8 + 2)) * dim
    out["sparse_c3"] = {"workload": "C3: 2^28-dim dense fp32, 10 % nnz, 256 bins, 8 groups, 2 rows, colRatio 0.3",
                        "nnz": nnz, "encode_ms": round(te * 1e3, 3), "gbps_dense_in": round(4.0 * dim / te / 1e9, 1),
                        "roofline_frac": round(alg / te / 1e9 / HBM_PEAK_GBS, 4), "restore_ms": round(td * 1e3, 3),
                        "note": "median wall time of 5 synchronised calls (one nnz read after the compaction, one read-back at the end)",
                        "parity_test": "tests/test_gpu_sparse_full.py::test_c3_full_size_matches_oracle"}
    del d, rk, rv
    out["sparse_aggregate"] = sparse_aggregate(sk, spl, dim, timed_median, dev)
    out["sparse_aggregate"]["parity_test"] = \
        "tests/test_gpu_sparse_exchange.py::test_decode_sum_eight_distinct_c3_payloads_full_size"
    return out


def c3_dense(dev, seed, dim=2**28):
    """A C3-shaped dense gradient: N(0, 1), 10 % of the entries kept; rank r's is seed 3 + r."""
    g = torch.Generator(device=dev).manual_seed(seed)
    d = torch.randn(dim, device=dev, generator=g)
    d[torch.rand(dim, device=dev, generator=g) >= 0.1] = 0.0
    return d


def sparse_aggregate(sk, spl, dim, timed_median, dev, P=8):
    """The ml path's DP step after the all-gather: P exported C3 payloads in
    stride-spaced slots -> Gradient.sum in double on the device (skml_sparse_decode_sum_f64), plus
    the export itself.  The P payloads are distinct, as in the DP step: rank r's C3 gradient
    (dense seed 3 + r, the sparse_exchange_step data) encoded with seeds 3 + r; their keys cover
    ~57 % of the dims.  tests/test_gpu_sparse_exchange.py checks this exact sum against the oracle."""
    from sketchml_amd.distributed import blob_stride
    pls = [spl]
    for r in range(1, P):
        d = c3_dense(dev, 3 + r, dim)
        pls.append(sk.encode_dense_as_sparse(d, 256, 8, 2, 0.3, 3 + r, 3 + r))
        del d
    sizes = [p.export_bytes() for p in pls]
    stride = blob_stride(sizes)
    allb = torch.zeros(stride * P, dtype=torch.uint8, device="cuda")
    tx, _ = timed_median(lambda: spl.export(allb[:stride]), 5)
    for q in range(1, P):
        pls[q].export(allb[q * stride:(q + 1) * stride])
    out = torch.empty(dim, dtype=torch.float64, device="cuda")
    ts, _ = timed_median(lambda: sk.decode_sum(allb, P, stride, dim, 1.0 / P, out), 5)
    t1, _ = timed_median(lambda: sk.decode_sum(allb, 1, stride, dim, 1.0, out), 5)
    nnz = [p.nnz() for p in pls]
    # algorithmic bytes: every blob read once, the 2^28 double sum written once
    alg = float(sum(sizes)) + 8.0 * dim
    res = {"workload": f"Gradient.sum of {P} distinct C3 sparse payloads (dense seeds 3..{2 + P}, nnz {min(nnz)}.."
                       f"{max(nnz)}) into a 2^28-dim double sum, x 1/{P}",
           "blob_bytes": sizes, "export_ms": round(tx * 1e3, 3), "decode_sum_ms": round(ts * 1e3, 3),
           "decode_sum_one_payload_ms": round(t1 * 1e3, 3),
           "per_payload_ms": round((ts - t1) / (P - 1) * 1e3, 3),
           "alg_bytes": alg, "roofline_frac": round(alg / ts / 1e9 / HBM_PEAK_GBS, 4),
           "note": "8 distinct payloads; median wall time of 5 synchronised calls; one payload = DeltaAdaptive "
                   "decode + MinMax query (restores alternate between two streams) + add into the double sum tile "
                   "by tile in payload order; the fixed part is the 2 GiB write of the sum (the x 1/P scale is fused "
                   "into it); alg_bytes = P blobs read + the sum written"}
    del allb, out, pls
    return res


def dense_decode_sum(sk, lib, ctx, dev, n, bins, seed0, P=8):
    """C4's consumer on one GPU: P = 8 gathered 2^26-value dense payloads (bucket r drawn with
    generator seed seed0 + r, encoded with params seed seed0) -> fused decode + sum in double +
    x 1/P (skml_dense_decode_sum_f32), HIP-event timed on the codec stream.  Algorithmic bytes =
    P * n * b / 8 (codes) + 4 n (fp32 out).  With bins = 4 and n = 2^27: C5's consumer (each rank
    sums the 8 gathered 2^27-float shards' 2-bit payloads)."""
    gen = torch.Generator(device=dev)
    xs = []
    for r in range(P):
        gen.manual_seed(seed0 + r)
        xs.append(torch.randn(n, device=dev, generator=gen))
    p = _lib_params(bins)
    p.seed = seed0
    nb = lib.skml_dense_payload_bytes(n, bins)
    stride = (nb + 255) // 256 * 256
    allp = sk.alloc_aligned(stride * P, dev)
    ptrs = (C.c_void_p * P)(*[xs[i % len(xs)].data_ptr() for i in range(P)])
    pptr = (C.c_void_p * P)(*[allp.data_ptr() + i * stride for i in range(P)])
    ns = (C.c_int64 * P)(*([n] * P))
    caps = (C.c_size_t * P)(*([stride] * P))
    if lib.skml_dense_encode_batch_f32(ctx, P, ptrs, ns, C.byref(p), pptr, caps):
        raise RuntimeError("batch encode failed")
    torch.cuda.synchronize()
    del xs
    out = torch.empty(n, dtype=torch.float32, device=dev)
    run = lambda: lib.skml_dense_decode_sum_f32(ctx, C.c_void_p(allp.data_ptr()), P, stride,  # noqa: E731
                                                 C.c_void_p(out.data_ptr()), n, 1.0 / P)
    run()
    torch.cuda.synchronize()
    lib.skml_ctx_set_timing(ctx, 1 << 5)
    lib.skml_ctx_reset_stats(ctx)
    for _ in range(10):
        run()
    ks = kernel_stats(lib, ctx)
    lib.skml_ctx_set_timing(ctx, 0)
    hdr = _lib_header(lib, ctx, allp)
    us = ks["k_decode_sum"]["avg_us"]
    alg = P * n * hdr.code_bits / 8.0 + 4.0 * n
    del allp, out
    return {"workload": f"{P} dense payloads of 2^{n.bit_length() - 1} codes ({hdr.code_bits}-bit, {hdr.bin_num} bins) "
                        f"-> one fp32 sum x 1/{P}",
            "k_decode_sum_us": round(us, 2), "alg_bytes": alg,
            "gbps": round(alg / (us * 1e-6) / 1e9, 1), "roofline_frac": round(alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}


def dense_bucket(sk, lib, ctx, dev, xs, label, bins=256, reps=50):
    """One dense configuration (rotating device buckets `xs`) outside the headline: encode time =
    mean of `reps` back-to-back encodes between two synchronisations; the per-kernel split comes
    from HIP events on the codec stream in a separate pass."""
    n = xs[0].numel()
    nb = lib.skml_dense_payload_bytes(n, bins)
    pl = sk.alloc_aligned(nb, dev)
    p = _lib_params(bins)
    p.seed = 2

    def enc(i):
        st = lib.skml_dense_encode_f32(ctx, C.c_void_p(xs[i % len(xs)].data_ptr()), n, C.byref(p),
                                       C.c_void_p(pl.data_ptr()), nb)
        if st:
            raise RuntimeError("encode failed")

    for i in range(5):
        enc(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        enc(i)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    lib.skml_ctx_set_timing(ctx, -1)
    lib.skml_ctx_reset_stats(ctx)
    for i in range(10):
        enc(i)
    ks = kernel_stats(lib, ctx)
    lib.skml_ctx_set_timing(ctx, 0)
    hdr = _lib_header(lib, ctx, pl)
    alg = (8.0 + hdr.code_bits / 8.0) * n
    res = {"workload": label, "ms": round(t * 1e3, 4),
           "gbps_fp32_in": round(4.0 * n / t / 1e9, 1), "roofline_frac_9B": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
           "bin_num_effective": hdr.bin_num,
           "kernels_us": {k: round(v["avg_us"], 2) for k, v in ks.items()}}
    if "k_leaf" in ks:
        res["k_leaf_gbps"] = round(4.0 * n / (ks["k_leaf"]["avg_us"] * 1e-6) / 1e9, 1)
    if "k_quantize" in ks:
        q = ks["k_quantize"]["avg_us"] * 1e-6
        res["k_quantize_gbps"] = round((4.0 + hdr.code_bits / 8.0) * n / q / 1e9, 1)
    del pl
    return res


def sparse_exchange_step(sk, exch, dev, rank, world, barrier, reps=3):
    """The ml path's exchange at C3 shape on every rank (GeneralizedLinearModel.scala:145-156):
    rank r encodes its own 2^28-dim, 10 %-nnz gradient (seed 3 + r), then sizes are all-gathered,
    the blob is exported into its padded slot, the slots are all-gathered over RCCL and every rank
    computes Gradient.sum x 1/P in double.  Max over ranks of the median of `reps` steps."""
    from sketchml_amd import distributed as D
    dim = 2**28
    d = c3_dense(dev, 3 + rank, dim)
    spl = sk.encode_dense_as_sparse(d, 256, 8, 2, 0.3, 3 + rank, 3 + rank)
    del d
    nb = spl.export_bytes()
    ts, tg = [], []
    for _ in range(reps):
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stride = D.blob_stride(D.agree_sizes(nb))
        local = torch.empty(stride, dtype=torch.uint8, device=dev)
        spl.export(local)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        allb = D.gather_blobs(local, stride, exchange=exch)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        avg = sk.decode_sum(allb, world, stride, dim, 1.0 / world)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        ts.append(t3 - t0)
        tg.append(t2 - t1)
        del allb, avg, local
    t = torch.tensor([statistics.median(ts), statistics.median(tg)], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    step, gat = float(t[0].item()), float(t[1].item())
    algbw = world * stride / gat / 1e9
    return {"workload": "C3-shape sparse gradient per rank: sizes + export + RCCL all-gather of the padded blobs "
                        "+ Gradient.sum x 1/P in double on every rank",
            "blob_bytes_rank0": nb, "stride": stride, "step_ms": round(step * 1e3, 3),
            "allgather_ms": round(gat * 1e3, 3), "allgather_busbw_gbs": round(algbw * (world - 1) / world, 1)}


def _lib_header(lib, ctx, payload):
    from sketchml_amd import _lib
    hdr = _lib.DenseHeader()
    lib.skml_dense_info(ctx, C.c_void_p(payload.data_ptr()), C.byref(hdr), None, 0)
    return hdr


def host_path_rates(lib, ctx, x, n, params, reps=5):
    """fp32-in GB/s of skml_dense_encode_host_f32 (host gradient -> device -> encode -> payload
    bytes back in host memory, synchronous), from pageable memory (a numpy array, as a JVM
    float[] pinned by GetPrimitiveArrayCritical is) and from skml_host_alloc pinned memory (a Java
    direct ByteBuffer), plus the PCIe copy rates alone for the same byte counts."""
    from sketchml_amd import _lib
    host = x.cpu().numpy()
    cap = lib.skml_dense_payload_bytes(n, params.bin_num)
    out = np.zeros(cap, dtype=np.uint8)
    wrote = C.c_size_t()
    res = {}

    def run(src_ptr, dst_ptr):
        st = lib.skml_dense_encode_host_f32(ctx, src_ptr, n, C.byref(params), dst_ptr, cap, C.byref(wrote))
        if st:
            raise RuntimeError(_lib.last_error())
        t0 = time.perf_counter()
        for _ in range(reps):
            lib.skml_dense_encode_host_f32(ctx, src_ptr, n, C.byref(params), dst_ptr, cap, C.byref(wrote))
        return (time.perf_counter() - t0) / reps

    t = run(host.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p))
    res["pageable"] = {"ms": round(t * 1e3, 3), "gbps_fp32_in": round(4.0 * n / t / 1e9, 2)}
    px, pp = C.c_void_p(), C.c_void_p()
    if lib.skml_host_alloc(4 * n, C.byref(px)) == 0 and lib.skml_host_alloc(cap, C.byref(pp)) == 0:
        np.ctypeslib.as_array(C.cast(px, C.POINTER(C.c_float)), shape=(n,))[:] = host
        t = run(px, pp)
        res["pinned"] = {"ms": round(t * 1e3, 3), "gbps_fp32_in": round(4.0 * n / t / 1e9, 2)}
        # the PCIe floor for the same bytes: H2D of the input + D2H of the payload, pinned
        pin_x = torch.from_numpy(host).pin_memory()
        d = torch.empty(n, dtype=torch.float32, device="cuda")
        pin_o = torch.empty(wrote.value, dtype=torch.uint8).pin_memory()
        do = torch.empty(wrote.value, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            d.copy_(pin_x, non_blocking=True)
            pin_o.copy_(do, non_blocking=True)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        res["pcie_copies_only"] = {"ms": round(t * 1e3, 3), "gbps_fp32_in": round(4.0 * n / t / 1e9, 2)}
    lib.skml_host_free(px)
    lib.skml_host_free(pp)
    res["payload_bytes"] = wrote.value
    return res


def _workload_label(args, world):
    """config.workload from the run's own arguments (BASELINE configs named where they match)."""
    n, bins = args.n, args.bins
    npow = f"2^{n.bit_length() - 1}" if n & (n - 1) == 0 else str(n)
    tag = ""
    if (args.quant, args.dtype) == ("quantile", "f32"):
        if n == 2**28 and bins == 256:
            tag = "north star: "
        elif n == 2**26 and bins == 256:
            tag = "C4: " if world > 1 else "C2: "
        elif n == 2**27 and bins == 4 and world > 1:
            tag = "C5 shard: "
    kind = "" if (args.quant, args.dtype) == ("quantile", "f32") else f"{args.quant} quantizer, {args.dtype} input, "
    return (f"{tag}{npow}-{'double' if args.dtype == 'f64' else 'float'} dense gradient bucket per GPU, "
            f"{bins} requested bins, {kind}encode" + (" + RCCL all-gather of payloads" if world > 1 else ""))


def _lib_params(bins):
    from sketchml_amd import _lib
    p = _lib.Params()
    _lib.lib.skml_params_default(C.byref(p))
    p.bin_num = bins
    return p


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return None


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))  # one process per GPU, started before any GPU call
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        return dry_run(args, world, rank)
    # SKML_BENCH_EXCHANGE=1 runs the N > 1 exchange path (RCCL all-gather on its own stream) with a
    # world-size-1 communicator: a one-GPU rehearsal of the code the multi-GPU runs take
    rehearse = world == 1 and os.environ.get("SKML_BENCH_EXCHANGE") == "1"
    if world > 1 or rehearse:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import sketchml_amd as sk
    from sketchml_amd import _lib
    lib = _lib.lib
    ctx = sk.get_context(dev.index).handle

    n, bins = args.n, args.bins
    nb = lib.skml_dense_payload_bytes(n, bins)
    esize = 8 if args.dtype == "f64" else 4
    # rotating buckets: at least 2, and at least 1 GiB in all, so no step starts on bytes the
    # previous step left in the 256 MB Infinity Cache
    nbuf = args.buffers if args.buffers > 0 else max(2, -(-(2**30) // (esize * n)))
    gen = torch.Generator(device=dev)
    xs = []
    for b in range(nbuf):
        # rank r's first bucket is seeded 6 + r (rank 0: the data of
        # tests/test_gpu_configs.py::test_north_star_2p28_matches_oracle)
        gen.manual_seed(6 + rank + 1000 * b)
        xs.append(torch.randn(n, device=dev, generator=gen,
                              dtype=torch.float64 if args.dtype == "f64" else torch.float32))
    payload = sk.alloc_aligned(nb, dev)
    params = _lib.Params()
    lib.skml_params_default(C.byref(params))
    params.bin_num = bins
    params.seed = 6 + rank

    exch = None
    allp = None
    payloads = [payload]
    if world > 1 or rehearse:
        from sketchml_amd.distributed import PayloadExchange
        # The exchange runs on its own stream and context, so step i's all-gather overlaps step
        # i + 1's encode (the gradient buckets of one DDP step are independent): two payload
        # buffers, each reused only after its previous all-gather has read it.
        ex_stream = torch.cuda.Stream(dev)
        with torch.cuda.stream(ex_stream):
            ex_ctx_obj = sk.Context(dev.index)  # bound to ex_stream at creation
        exch = PayloadExchange(ex_ctx_obj._h)  # RCCL communicator; unique id broadcast over the group
        allp = sk.alloc_aligned(nb * world, dev)
        payloads.append(sk.alloc_aligned(nb, dev))
        ev_enc = [torch.cuda.Event(), torch.cuda.Event()]
        ev_ex = [torch.cuda.Event(), torch.cuda.Event()]
        ex_used = [False, False]
        main_stream = torch.cuda.current_stream(dev)

    encode = getattr(lib, {("quantile", "f32"): "skml_dense_encode_f32",
                           ("quantile", "f64"): "skml_dense_encode_f64",
                           ("uniform", "f32"): "skml_dense_encode_uniform_f32",
                           ("uniform", "f64"): "skml_dense_encode_uniform_f64"}[(args.quant, args.dtype)])

    skip_exchange = [False]  # the N > 1 encode-only region (extras.encode_only)

    def step(i):
        x = xs[i % nbuf]
        b = i % len(payloads)
        if skip_exchange[0]:
            st = encode(ctx, C.c_void_p(x.data_ptr()), n, C.byref(params), C.c_void_p(payloads[b].data_ptr()), nb)
            if st:
                raise RuntimeError(_lib.last_error())
            return
        if exch is not None and ex_used[b]:
            main_stream.wait_event(ev_ex[b])  # the previous all-gather of this buffer has read it
        p = payloads[b]
        st = encode(ctx, C.c_void_p(x.data_ptr()), n, C.byref(params), C.c_void_p(p.data_ptr()), nb)
        if st:
            raise RuntimeError(_lib.last_error())
        if exch is not None:
            ev_enc[b].record(main_stream)
            ex_stream.wait_event(ev_enc[b])
            exch.allgather(p, nb, allp)
            ev_ex[b].record(ex_stream)
            ex_used[b] = True

    def barrier():
        if dist.is_initialized():
            dist.barrier()

    # warm-up: W untimed steps, continued until --warmup-ms of wall time has passed.  The engine
    # clock needs ~25 ms of sustained load to settle: in a kernel trace of the first 85 encodes
    # (profiles/r05b_warmup_ramp.txt) the leaf runs 400-445 us for the first ten and settles at
    # ~340 us after ~40; five steps (3 ms) leave the timed region inside that ramp.
    # Every rank runs the same number of steps (each step may hold a collective).
    t_w = time.perf_counter()
    nwarm = max(1, args.warmup)
    for i in range(nwarm):
        step(i)
    torch.cuda.synchronize()
    el_ms = (time.perf_counter() - t_w) * 1e3
    extra = 0 if el_ms >= args.warmup_ms else int(np.ceil((args.warmup_ms - el_ms) / (el_ms / nwarm)))
    if world > 1:
        t = torch.tensor([extra], device=dev, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        extra = int(t.item())
    for i in range(extra):
        step(nwarm + i)
    nwarm += extra
    torch.cuda.synchronize()

    def timed_region(first):
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(first + i)
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # the headline: K encodes, nothing else on the stream
    elapsed = timed_region(nwarm)
    # the same K encodes again with HIP events around the leaf launches only (on the codec
    # stream): the live kernel time of the roofline, measured outside the headline's region
    lib.skml_ctx_set_timing(ctx, 1 << 0)
    lib.skml_ctx_reset_stats(ctx)
    elapsed_ev = timed_region(nwarm + args.steps)
    lib.skml_ctx_set_timing(ctx, 0)
    kstats = kernel_stats(lib, ctx)
    # per-kernel breakdown of the whole encode (every kernel timed) in a separate, untimed pass
    lib.skml_ctx_set_timing(ctx, -1)
    lib.skml_ctx_reset_stats(ctx)
    for i in range(min(args.steps, 10)):
        step(i)
    torch.cuda.synchronize()
    lib.skml_ctx_set_timing(ctx, 0)
    allstats = kernel_stats(lib, ctx)
    steps_b = min(args.steps, 10)

    ms_per_step = 1000.0 * elapsed / args.steps
    value = world * esize * n * args.steps / elapsed / 1e9

    # ---- roofline of the dominant kernel (algorithmic bytes per launch / avg duration) ----
    hdr = _lib.DenseHeader()
    lib.skml_dense_info(ctx, C.c_void_p(payload.data_ptr()), C.byref(hdr), None, 0)
    code_bits = hdr.code_bits
    alg_bytes = {"k_leaf": esize * n, "k_quantize": esize * n + n * code_bits / 8.0,
                 "k_merge": esize * 128 * max(1, n // 256 // 64),
                 # the uniform quantizer's min/max pass reads the bucket once (k_uni_minmax + finish)
                 "k_summary": esize * n if args.quant == "uniform" else 0.0}
    # dominant kernel by device time in the full breakdown; its duration from the live timed region
    dom = max((k for k in allstats if k in alg_bytes), key=lambda k: allstats[k]["avg_us"] * allstats[k]["launches"])
    live = kstats.get(dom, allstats[dom])
    ach = alg_bytes[dom] / (live["avg_us"] * 1e-6) / 1e9
    traffic = pmc_traffic(dom, n, args.dtype, args.quant)
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": traffic[0] if traffic else None,
                "traffic_source": traffic[1] if traffic else None,
                "alg_bytes_per_launch": alg_bytes[dom]}
    valu = sq_valu(dom, args.n) if (args.dtype == "f32" and args.quant == "quantile") else None
    if valu:
        # the sort-dominated leaf is bound by VALU issue, not HBM: its issue rate against the ceiling
        rate = valu[0] / (live["avg_us"] * 1e-6) / 1e9
        roofline["valu"] = {"insts_per_launch": valu[0], "source": valu[1], "issue_ginst_s": round(rate, 1),
                            "peak_ginst_s": round(VALU_PEAK_GINST, 1), "frac": round(rate / VALU_PEAK_GINST, 4),
                            "peak_source": ["profiles/r06_ubench_issue.txt", VALU_MIX_SOURCE],
                            "peak_note": f"one wave-instruction per clock per CU at 2.4 GHz (the measured rate "
                                         f"of the network's min / max / med3 / DPP ops: 4 SIMD cycles each) x "
                                         f"{VALU_MIX_FACTOR} for the leaf's share of 2-cycle adds, ands and "
                                         f"shifts (SIMD-32 rate)"}
    encode_device_us = sum(v["avg_us"] * v["launches"] for k, v in allstats.items()
                           if k in alg_bytes) / steps_b
    extras = {"encode_device_us": round(encode_device_us, 2),
              "encode_roofline_frac": round((2 * esize + code_bits / 8.0) * n / (encode_device_us * 1e-6)
                                            / 1e9 / HBM_PEAK_GBS, 4),
              "kernels": {k: {"avg_us": round(v["avg_us"], 2), "launches": v["launches"]}
                          for k, v in allstats.items()},
              "kernel_breakdown_note": f"every kernel event-timed over {steps_b} extra encodes outside "
                                       "the timed region; the roofline's live time comes from a second region of "
                                       "the same K encodes with events around the leaf only",
              "ms_per_step_leaf_evented": round(1000.0 * elapsed_ev / args.steps, 4),
              "warmup_steps_run": nwarm,
              "bin_num_effective": hdr.bin_num, "code_bits": code_bits}

    # ---- decode throughput + decode L2 error (rank-local) ----
    if not args.no_extras:
        out = torch.empty(n, dtype=xs[0].dtype, device=dev)
        decode = lib.skml_dense_decode_f64 if args.dtype == "f64" else lib.skml_dense_decode_f32
        x = xs[0]
        step(0)  # the payload decoded below is the encode of exactly this bucket
        lib.skml_ctx_set_timing(ctx, 1 << 4)
        lib.skml_ctx_reset_stats(ctx)
        for _ in range(10):
            decode(ctx, C.c_void_p(payload.data_ptr()), C.c_void_p(out.data_ptr()), n)
        dstats = kernel_stats(lib, ctx)
        lib.skml_ctx_set_timing(ctx, 0)
        dus = dstats["k_decode"]["avg_us"]
        diff = (out.double() - x.double())
        l2 = float(torch.linalg.vector_norm(diff).item())
        extras["decode"] = {"gbps_out": round(esize * n / (dus * 1e-6) / 1e9, 1), "avg_us": round(dus, 2),
                            "roofline_frac": round((esize + code_bits / 8.0) * n / (dus * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        extras["decode_l2_err"] = l2
        extras["decode_rmse"] = l2 / np.sqrt(n)
        extras["decode_rel_l2"] = l2 / float(torch.linalg.vector_norm(x.double()).item())
        # end-to-end with PCIe through the host entry point (the JNI path): host float[] ->
        # skml_dense_encode_host_f32 -> payload bytes in host memory
        if rank == 0 and args.dtype == "f32" and args.quant == "quantile":
            extras["host_path"] = host_path_rates(lib, ctx, x, n, params)
            extras["h2d_d2h_inclusive_gbps"] = extras["host_path"]["pageable"]["gbps_fp32_in"]

    # ---- N > 1: the same K encodes without the exchange (every rank's encode alone, at the max
    # over ranks), so the scaling line shows the encode's own weak scaling beside `value` ----
    if exch is not None:
        skip_exchange[0] = True
        el_enc = timed_region(nwarm + 2 * args.steps)
        skip_exchange[0] = False
        extras["encode_only"] = {"ms_per_step": round(1000.0 * el_enc / args.steps, 4),
                                 "value_gbps": round(world * esize * n * args.steps / el_enc / 1e9, 2),
                                 "note": "the same K steps with the payload all-gather left out; `value` keeps it "
                                         "(each step's all-gather overlaps the next step's encode)"}
    # ---- N > 1: the exchange step alone, and a check of the gathered payloads ----
    if exch is not None and not args.no_extras:
        from sketchml_amd.distributed import decode_sum
        reps = 10
        barrier()
        torch.cuda.synchronize()
        ta = time.perf_counter()
        for _ in range(reps):
            exch.allgather(payload, nb, allp)
        torch.cuda.synchronize()
        tag = (time.perf_counter() - ta) / reps
        t = torch.tensor([tag], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tag = float(t.item())
        algbw = world * nb / tag / 1e9
        # fused decode + sum + 1/P of all gathered payloads vs the all-reduce of each rank's decode
        summed = torch.empty(n, dtype=torch.float32, device=dev)
        decode_sum(ctx, allp, world, nb, n, 1.0 / world, summed)
        own = torch.empty(n, dtype=torch.float32, device=dev)
        lib.skml_dense_decode_f32(ctx, C.c_void_p(payload.data_ptr()), C.c_void_p(own.data_ptr()), n)
        ref = own.double()
        dist.all_reduce(ref)
        err = float((summed.double() - ref / world).abs().max().item())
        extras["allgather"] = {"ms": round(tag * 1e3, 3), "bytes_per_rank": nb, "algbw_gbs": round(algbw, 1),
                               "busbw_gbs": round(algbw * (world - 1) / world, 1),
                               "decode_sum_max_abs_err_vs_allreduce": err}
        del summed, own, ref
        extras["sparse_exchange"] = sparse_exchange_step(sk, exch, dev, rank, world, barrier)

    if (rank == 0 and world == 1 and not args.no_extras and not args.no_configs and args.quant == "quantile"
            and args.dtype == "f32" and args.n == 2**28):
        extras["other_configs"] = other_configs(sk, lib, ctx, dev)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline and args.quant == "quantile" and args.dtype == "f32":
        # after every timed GPU region (the other ranks wait at the barrier below)
        cpu = cpu_baseline(xs[0][: 2**24].cpu().numpy(), bins, args.cpu_seconds)

    barrier()
    if exch is not None:
        exch.close()
    if rank == 0:
        line = {
            "metric": "device-resident grad encode GB/s (fp32 in) + decode L2 err, 1/2/4/8 GPU",
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "warmup_steps_run": nwarm, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "warmup_note": f"{nwarm} untimed encodes: --warmup {args.warmup}, extended to {args.warmup_ms:g} ms of "
                           "sustained load so the engine clock has settled (profiles/r05b_warmup_ramp.txt)",
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic N(0,1), torch generator",
            "config": {"workload": _workload_label(args, world),
                       "n_per_gpu": n, "bins": bins, "rotating_buffers": nbuf, "parallelism": f"dp{world}"},
            "roofline": roofline, "cpu_baseline": cpu, "extras": extras,
        }
        print(json.dumps(line))
    if exch is not None:
        exch.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
