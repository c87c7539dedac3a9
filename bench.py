#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): DM trials/s at 2^23 samples, P = 0.1-10 s.

Workload = BASELINE config 2: series of 2^23 float32
samples at 256 us, dereddened (running median 4 s, 101 points) and normalised,
then the full FFA periodogram over 0.1-10 s with 240-260 phase bins and 6
boxcar widths (1153 FFA transforms, L = 5,307,626 trial periods).  One "step"
= one batch of `--batch` DM trials per GPU, resident in HBM when the timed
region starts; the S/N array stays in HBM.  Trials are independent: each rank
processes its own batch (weak scaling, no data-path collective).

Prints one JSON line (rank 0).  Launch for N>1:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "DM trials/sec (node) at 2^23 samples, P=0.1-10 s; FFA-pass HBM GB/s"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CFG = dict(n=1 << 23, tsamp=256e-6, pmin=0.1, pmax=10.0, bmin=240, bmax=260, ducy_max=0.05,
           rmed_width=4.0, rmed_minpts=101)


def synth_batch(torch, B, n, tsamp, seed, device):
    """B synthetic DM trials on the device: white noise, a slow red-noise ramp,
    and a top-hat pulsar (P = 3.3 s, 2% duty cycle, amplitude 14) in trial 0."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn((B, n), generator=g, device=device, dtype=torch.float32)
    t = torch.arange(n, device=device, dtype=torch.float64) * tsamp
    ramp = (0.5 * torch.sin(2 * 3.141592653589793 * t / 700.0)).to(torch.float32)
    x += ramp
    on = torch.remainder(t / 3.3 + 0.3, 1.0) < 0.02
    x[0] += on.to(torch.float32) * (14.0 / float(on.sum().item()) ** 0.5)
    return x


def source_digest():
    """sha256 over the engine's kernel and host sources (riptide_amd/csrc):
    a PMC summary is only valid for the exact code it was measured on (there
    is no .git on the GPU box, so the check is by content, not by commit)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(REPO, "riptide_amd", "csrc", "*"))):
        if f.endswith((".hip", ".cpp", ".hpp", ".h", "Makefile")):
            h.update(os.path.basename(f).encode())
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic():
    """HBM bytes per trial of the cone kernel from the newest committed PMC
    summary (profiles/*_pmc_cone.json, written by tools/pmc_to_json.py from
    rocprofv3 FETCH_SIZE/WRITE_SIZE passes).  Returns (summary or None,
    reason): a summary measured on other kernel sources than these
    (`csrc_sha` != source_digest()) is stale and not used."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_cone.json")))   # r01a < r01b < ...: newest last
    if not files:
        return None, "no PMC summary under profiles/"
    with open(files[-1]) as f:
        d = json.load(f)
    src = os.path.relpath(files[-1], REPO)
    cur = source_digest()
    if d.get("csrc_sha") != cur:
        return None, (f"stale: {src} was measured on kernel sources {d.get('csrc_sha') or d.get('commit')}, "
                      f"these are {cur}")
    return {"hbm_bytes_per_trial": d["hbm_bytes_per_trial"], "source": src, "commit": d.get("commit")}, "ok"


def cpu_baseline(timeout_s=300):
    cmd = [sys.executable, os.path.join(REPO, "oracle", "cpu_baseline.py")]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, check=True).stdout
        res = json.loads(out.strip().splitlines()[-1])
        res.pop("seconds", None)
        return res
    except Exception as e:  # reported, never fatal for the GPU measurement
        return {"value": None, "unit": "DM trials/s", "cores": None, "kind": "reference", "sample": f"failed: {e}"}


def bench_cfg5(args, torch, dist, world, rank, local, dev):
    """BASELINE configs[4] (cfg5): SIGPROC .tim DM trials of 2^23 samples @ 64 us
    searched from files to peak lists, the rffa search stage
    (pipeline.py:177-189 with worker_pool.py:47-70) on the GPU worker pool:
    file read + H2D (8-bit files converted on the device) + deredden +
    normalise + 3 search ranges (example.yaml) + device peak detection, in
    DMIterator chunks.  Each rank searches its own files (weak scaling)."""
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import inputs
    from riptide_amd.reading import write_sigproc
    from riptide_amd.worker_pool import GpuWorkerPool, iterate_chunks
    c = inputs.CFG5
    tmp = tempfile.mkdtemp(prefix=f"cfg5_r{rank}_", dir=os.environ.get("TMPDIR", "/tmp"))
    fnames = []
    for j in range(args.files):
        k = rank * args.files + j
        data, hdr = inputs.cfg5_trial(k % 64)
        fn = os.path.join(tmp, f"DM{hdr['refdm']:08.2f}_{k:05d}.tim")
        write_sigproc(fn, data, hdr)
        fnames.append(fn)
    pool = GpuWorkerPool(c["dereddening"], c["ranges"], processes=args.batch, fmt="sigproc", batch=args.batch,
                         device=local)
    pool.process_fname_list(fnames[:args.batch])          # warmup: plans, device buffers
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    npeaks = 0
    for chunk in iterate_chunks(fnames, chunksize=args.batch):
        npeaks += len(pool.process_fname_list(chunk))
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    for fn in fnames:
        os.remove(fn)
    os.rmdir(tmp)
    if rank == 0:
        trials = world * args.files
        print(json.dumps({
            "metric": "DM trials/sec files->peaks (cfg5 rffa search stage, 2^23 samples @ 64 us, 3 ranges)",
            "value": trials / elapsed, "unit": "DM trials/s", "n_gpus": world, "steps": 1, "warmup": 1,
            "ms_per_step": elapsed * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic SIGPROC files (tests/golden/inputs.py cfg5_trial; 6 of 8 float32, "
                                    "2 of 8 8-bit) written to local disk before the timed region",
            "config": {"workload": "cfg5: rffa search stage on SIGPROC .tim files (example.yaml ranges short / "
                                   "medium / long, smin 6), DMIterator chunks of --batch files",
                       "files_per_gpu": args.files, "chunk": args.batch, "peaks_found": npeaks,
                       "parallelism": f"dm-trials x{world} (independent, weak scaling)"},
        }), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=16, help="DM trials per GPU per step")
    ap.add_argument("--workload", choices=("cfg2", "cfg5"), default="cfg2",
                    help="cfg2: headline periodogram throughput (device-resident); cfg5: files -> peaks")
    ap.add_argument("--files", type=int, default=32, help="cfg5: SIGPROC files per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    # transform-group scratch per ping/pong buffer and trial (capi.cpp
    # scratch_budget_floats): 384 M floats = 26 instead of 94 cone launches per
    # step, ~1 % faster (tools/ab_sched.py); 49 GB of the 288 GB HBM at 16 trials
    if args.workload == "cfg2":
        os.environ.setdefault("RIPTIDE_AMD_SCRATCH_MFLOATS", "384")
    import torch
    import torch.distributed as dist
    from riptide_amd import engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if args.workload == "cfg5":
        bench_cfg5(args, torch, dist, world, rank, local, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    c = CFG
    plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"], device=local)
    B = args.batch
    ws_samples = int(round(c["rmed_width"] / c["tsamp"]))
    raw = synth_batch(torch, B, c["n"], c["tsamp"], 1000 + rank, dev)
    xbuf = torch.empty_like(raw)
    dws = torch.empty(engine.deredden_workspace_bytes(c["n"], ws_samples, c["rmed_minpts"], B),
                      dtype=torch.uint8, device=dev)
    snr = torch.empty((B, plan.length, plan.num_widths), dtype=torch.float32, device=dev)
    pws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device=dev)

    def step():
        engine.deredden_normalise(raw, ws_samples, c["rmed_minpts"], out=xbuf, workspace=dws)
        plan.run(xbuf, out=snr, workspace=pws)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    plan.check()                  # device error flag of the warmup runs
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    engine.profile_reset()
    engine.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    engine.profile_enable(False)
    plan.check()                  # every timed step: no unit refused (the flag is sticky)
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    cone = engine.profile_read(0)
    ladder = engine.profile_read(1)
    stats = plan.stats()

    if rank == 0:
        pmc, pmc_reason = pmc_traffic()
        trials = world * B * args.steps
        achieved = cone["alg_bytes"] / (cone["ms"] * 1e-3) / 1e9 if cone["ms"] > 0 else None
        line = {
            "metric": METRIC,
            "value": trials / elapsed,
            "unit": "DM trials/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device-generated white noise + red-noise ramp + top-hat pulsar; resident in HBM)",
            "config": {
                "workload": "cfg2: 2^23 samples @ 256 us, deredden(4 s, 101 pts) + normalise + FFA periodogram "
                            "P=0.1-10 s, bins 240-260, widths [1,2,3,4,6,9]",
                "trials_per_step_per_gpu": B,
                "trial_periods": plan.length,
                "ffa_transforms": stats["transforms"],
                "cone_launches_per_step": stats["launches"],
                "scratch_mfloats_per_buffer_trial": float(os.environ["RIPTIDE_AMD_SCRATCH_MFLOATS"]),
                "parallelism": f"dm-trials x{world} (independent, weak scaling)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "cone_kernel (FFA passes + fused boxcar S/N)",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": (pmc["hbm_bytes_per_trial"] * B / stats["launches"]) if pmc else None,
                "traffic_per_trial": pmc["hbm_bytes_per_trial"] if pmc else None,
                "traffic_source": pmc["source"] if pmc else None,
                "traffic_status": pmc_reason,
                "alg_bytes_per_launch": stats["alg_bytes"] * B / stats["launches"],
                "alg_bytes_per_trial": stats["alg_bytes"],
                "moved_bytes_per_trial": stats["moved_bytes"],
                "kernel_ms_per_step": cone["ms"] / args.steps,
                "kernel_launches_per_step": cone["launches"] / args.steps,
                "ladder_ms_per_step": ladder["ms"] / args.steps,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
