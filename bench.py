"""bench.py — sampled molecules/sec for the equivariant-CNF sample path (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): LJ13 (N = 13, D = 3, lj13.yaml network), batch 1024 molecules per GPU,
fixed-step ODE with NFE = 100 (Euler, dt = 0.01), fp32, synthetic inputs (x0 from the zero-CoM
base with a seeded draw) and flax-default random-init weights of the lj13 architecture.

One "step" = one full sample of the batch: x0 (resident in HBM) -> 100 EGNN evaluations -> x1, i.e. one
ecnf_integrate launch.  Multi-GPU: one process per GPU (torchrun), each rank samples its own 1024 molecules
(weak scaling, no data-path collective); the timing is the max over ranks.

Extra fields: "roofline" (dominant kernel = integrate_kernel, MFMA bound: algorithmic fp32 FLOPs per launch /
average launch time from HIP events on the launch stream, against the ceiling of the kernel's instruction mix —
GEMM FLOPs at the split-fp16 rate, vector FLOPs at the fp32 rate; see roofline_peak), "matmul" (which
arithmetic the GEMMs run) and "cpu_baseline" (the oracle's numpy fp32 batched
restatement of the same Euler solve on a bounded sample, rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
sys.path.insert(0, ROOT)

PEAK_FP32_MFMA_TFLOPS = 157.3    # MI355X dense FP32 matrix peak (MI355X_MICROARCH.md, chip-level parameters)
PEAK_16BIT_MFMA_TFLOPS = 2516.6  # MI355X dense BF16 = FP16 matrix peak: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz
SPLIT_TERMS = {"split_f16": 3, "split_bf16": 6}   # 16-bit cross terms per fp32 product (chain_split.hpp)


def flops_per_eval(cfg) -> float:
    """Dense-contraction FLOPs of one EGNN evaluation of one molecule with the phi_e layer-1 per-node
    factorisation: F = K [2N(H+T)H + 4NHM + 3EM + 2E(L-1)M^2 + 2ELM^2 + 4EM
    + 2N((M+H)M + (L-1)M^2 + MH)]."""
    N, H, T, M, L, K = cfg.n_nodes, cfg.hidden, cfg.time_embedding_dim, cfg.mlp_width, cfg.mlp_depth, cfg.n_blocks
    E = N * (N - 1)
    return K * (2 * N * (H + T) * H + 4 * N * H * M + 3 * E * M + 2 * E * (L - 1) * M * M + 2 * E * L * M * M
                + 4 * E * M + 2 * N * ((M + H) * M + (L - 1) * M * M + M * H))


def dead_flops_per_eval(cfg) -> float:
    """FLOPs of flops_per_eval that no output depends on: the last block's h update (gate dot 2EM and phi_h), since
    the field is x_K - x_c - mean(x) (egnn.py:176-188).  jit (XLA dead-code elimination) drops them in the reference
    and the kernel skips them, so the roofline counts live FLOPs only."""
    N, H, M, L = cfg.n_nodes, cfg.hidden, cfg.mlp_width, cfg.mlp_depth
    E = N * (N - 1)
    return 2 * E * M + 2 * N * ((M + H) * M + (L - 1) * M * M + M * H)


def live_flops_per_eval(cfg) -> float:
    return flops_per_eval(cfg) - dead_flops_per_eval(cfg)


def vector_flops_per_eval(cfg) -> float:
    """The part of live_flops_per_eval that is not a GEMM (runs on the fp32 VALU): phi_e layer-1 assembly (3EM), the
    phi_x-output dot product (2EM) and the gate dot product (2EM, every block but the last)."""
    N, M, K = cfg.n_nodes, cfg.mlp_width, cfg.n_blocks
    E = N * (N - 1)
    return K * (3 * E * M + 4 * E * M) - 2 * E * M


def roofline_peak(cfg, chain_mode: str) -> float:
    """Ceiling (TFLOP/s of algorithmic fp32 FLOPs) for this kernel's instruction mix.  Split modes run every GEMM
    (edge chain and node GEMMs) on the 16-bit matrix cores at (dense 16-bit peak / cross terms) and the vector
    FLOPs at the fp32 rate: peak = F / (F_gemm / P_split + F_vec / P_fp32); fp32_mfma: the fp32 MFMA peak."""
    F = live_flops_per_eval(cfg)
    if chain_mode not in SPLIT_TERMS:
        return PEAK_FP32_MFMA_TFLOPS
    Fv = vector_flops_per_eval(cfg)
    p_split = PEAK_16BIT_MFMA_TFLOPS / SPLIT_TERMS[chain_mode]
    return F / ((F - Fv) / p_split + Fv / PEAK_FP32_MFMA_TFLOPS)


def cpu_baseline(cfg_name: str, n_mol: int, nfe: int, threads: int):
    """Time the oracle (numpy fp32, batched like XLA's vmap) on `n_mol` molecules x `nfe` Euler steps."""
    import numpy as np
    from threadpoolctl import threadpool_limits
    from oracle import ecnf_oracle as O
    oc = O.CONFIGS[cfg_name]
    params = O.init_params(oc, 0)
    rng = np.random.default_rng(0)
    z = rng.standard_normal((n_mol, oc.n_nodes * oc.dim)).astype(np.float32)
    x0 = O.base_sample(z, oc)
    feat = np.zeros((n_mol, oc.n_nodes), np.int32)
    with threadpool_limits(limits=threads):
        O.sample_cnf(params, oc, x0[:2], feat[:2], solver="euler", dt0=0.5)   # warm-up
        t0 = time.perf_counter()
        O.sample_cnf(params, oc, x0, feat, solver="euler", dt0=1.0 / nfe)
        dt = time.perf_counter() - t0
    return n_mol / dt, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="molecules per GPU per step")
    ap.add_argument("--config", default="lj13")
    ap.add_argument("--nfe", type=int, default=100)
    ap.add_argument("--cpu-molecules", type=int, default=160, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) or gloo (multi-rank rehearsal)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    from ecnf_amd import CONFIGS, init_params
    from ecnf_amd.engine import EcnfHandle, SolveOptions

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev                      # one rank per GPU; folds ranks onto fewer GPUs only in rehearsals
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", local)
    cfg = CONFIGS[args.config]

    h = EcnfHandle(cfg, init_params(cfg, 0), local)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)                       # each rank samples its own molecules
    z = torch.randn((args.batch, cfg.event_dim), generator=g, device=dev)
    x0 = h.base_sample(z)
    feat = torch.zeros((args.batch, cfg.n_nodes), device=dev, dtype=torch.int32)
    opts = SolveOptions(solver="euler", step_size=1.0 / args.nfe)

    def step():
        return h.integrate(x0, feat, 0.0, 1.0, opts, check_status=False)

    for _ in range(args.warmup):
        y1, _, nfe, _ = step()
    torch.cuda.synchronize(dev)
    nfe_seen = int(nfe.max()) if args.warmup else args.nfe

    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        y1, _, nfe, status = step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t.item())
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    assert int((status != 0).sum()) == 0 and torch.isfinite(y1).all()

    value = world * args.batch * args.steps / t_max
    F = live_flops_per_eval(cfg)
    achieved = F * nfe_seen * args.batch / (kernel_ms * 1e-3) / 1e12
    chain_mode = h.chain_arithmetic()
    peak = roofline_peak(cfg, chain_mode)

    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.config}_b{args.batch}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")

    cpu = None
    if rank == 0 and world == 1 and args.cpu_molecules > 0:
        threads = args.cpu_threads or len(os.sched_getaffinity(0))
        rate, secs = cpu_baseline(args.config, args.cpu_molecules, args.nfe, threads)
        cpu = {"value": rate, "unit": "molecules/s", "cores": threads, "kind": "port",
               "sample": f"{args.cpu_molecules} LJ13 molecules x {args.nfe} Euler steps, oracle numpy fp32 "
                         f"batched restatement ({secs:.1f} s)"}

    if rank == 0:
        out = {
            "metric": "sampled molecules/sec (fixed-step ODE, NFE=100), LJ13 N=13",
            "value": value,
            "unit": "molecules/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded zero-CoM Gaussian x0, flax-default random-init lj13 weights)",
            "config": {"workload": f"{args.config} sample, Euler NFE={nfe_seen}, batch {args.batch}/GPU",
                       "n_nodes": cfg.n_nodes, "batch_per_gpu": args.batch, "global_batch": world * args.batch,
                       "nfe": nfe_seen, "solver": "euler", "parallelism": f"dp{world}"},
            "matmul": {"gemms": chain_mode, "tangent_kernels": f"{chain_mode} edge chains, fp32_mfma node GEMMs",
                       "accumulate": "f32"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": traffic,
                         "kernel": "integrate_kernel", "kernel_ms": kernel_ms,
                         "flop_per_launch": F * nfe_seen * args.batch,
                         "flop_basis": "live dense-contraction FLOPs per EGNN eval (SURVEY 8d F minus the last "
                                       "block's dead h update) x NFE x batch",
                         "frac_vs_fp32_mfma_peak": achieved / PEAK_FP32_MFMA_TFLOPS,
                         "peak_basis": (f"GEMM FLOPs at the dense 16-bit MFMA peak / {SPLIT_TERMS[chain_mode]} split "
                                        "terms, vector FLOPs at the fp32 peak") if chain_mode in SPLIT_TERMS
                                       else "fp32 MFMA peak"},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
