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
import math
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


def pmc_traffic(workload="cfg2"):
    """HBM bytes per trial of the cone kernel from the newest committed PMC
    summary of this workload (profiles/*_pmc_cone.json for cfg2,
    profiles/*_pmc_cone_<cfg>.json for the others; written by
    tools/pmc_to_json.py from rocprofv3 FETCH_SIZE/WRITE_SIZE passes).
    Returns (summary or None, reason): the newest summary measured on these
    kernel sources (`csrc_sha` == source_digest()); one measured on other
    sources is stale and not used."""
    import glob
    pat = "*_pmc_cone.json" if workload == "cfg2" else f"*_pmc_cone_{workload}.json"
    files = sorted(glob.glob(os.path.join(REPO, "profiles", pat)))   # r01a < r01b < ...: newest last
    if not files:
        return None, f"no {workload} PMC summary under profiles/"
    cur = source_digest()
    for fn in reversed(files):
        with open(fn) as f:
            d = json.load(f)
        if d.get("csrc_sha") == cur:
            return {"hbm_bytes_per_trial": d["hbm_bytes_per_trial"], "source": os.path.relpath(fn, REPO),
                    "commit": d.get("commit")}, "ok"
    with open(files[-1]) as f:
        d = json.load(f)
    return None, (f"stale: {os.path.relpath(files[-1], REPO)} (the newest) was measured on kernel sources "
                  f"{d.get('csrc_sha') or d.get('commit')}, these are {cur}; no summary matches")


def cpu_baseline(workload="cfg2", cores="", extra=(), timeout_s=400):
    cmd = [sys.executable, os.path.join(REPO, "oracle", "cpu_baseline.py"), "--workload", workload]
    if cores:
        cmd += ["--cores", str(cores)]
    cmd += list(extra)
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, check=True).stdout
        res = json.loads(out.strip().splitlines()[-1])
        res.pop("seconds", None)
        return res
    except Exception as e:  # reported, never fatal for the GPU measurement
        return {"value": None, "unit": "DM trials/s", "cores": None, "kind": "reference", "sample": f"failed: {e}"}


def cpu_baselines(workload, extra=()):
    """The rffa CPU model on this host: `cpu_baseline` on this process's CPU
    share (16 cores per GPU on the GPU box), plus `node` on every core this
    process may use (affinity mask capped by a cgroup CPU quota), each with
    its core count.  Where the host grants fewer cores than its affinity mask
    shows (a shared GPU box), `node_extrapolated` scales the measured
    per-core rate to the affinity cores -- labelled, not measured."""
    share = cpu_baseline(workload, extra=extra)
    aff = share.get("affinity_cores")
    quota = share.get("cpu_quota_cores")
    usable = min(aff, int(quota)) if (aff and quota) else aff
    if share.get("cores") and usable and usable > share["cores"]:
        share["node"] = cpu_baseline(workload, cores="all", extra=extra)
    else:
        share["node"] = {"same_as_share": True, "cores": share.get("cores")}
    node_cores = share["node"].get("cores") or 0
    if aff and share.get("per_core_search_per_s") and node_cores < aff:
        share["node_extrapolated"] = {
            "value": share["per_core_search_per_s"] * aff, "unit": "DM trials/s", "cores": aff,
            "basis": f"per-core rate of the {share.get('cores')}-core run x {aff} affinity cores; this host "
                     f"grants {quota if quota else node_cores} cores, so the node figure is extrapolated, "
                     f"not measured"}
    return share


def roofline(engine, cone, stats, trials_per_launch_unit, pmc=None, pmc_reason=None):
    """The roofline object of a bench line: Σ algorithmic bytes of the cone
    launches ÷ Σ their HIP-event durations, against 8 TB/s."""
    achieved = cone["alg_bytes"] / (cone["ms"] * 1e-3) / 1e9 if cone["ms"] > 0 else None
    B = trials_per_launch_unit
    return {
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
    }


def floor_bytes_per_trial(c, plan, stats):
    """SURVEY.md §8(d)'s implementation-independent floor of one trial's
    periodogram: every used rung reads the series and writes its downsampled
    series once (Σ_rungs 4N + 4n), every transform reads its input block once
    (4·Σ m·p = 4·cells), the S/N is written once (4·L·W) and the grid once
    (12·L: periods f64 + foldbins u32).  The rungs follow periodogram.hpp:
    135-175 (f = f0·g^k, n = floor(N / f), bstop = min(bmax, n, floor(pmax /
    tau)); a rung with bstop < bmin feeds no transform)."""
    n_in, tsamp = c["n"], c["tsamp"]
    f0 = c["pmin"] / (tsamp * c["bmin"])
    g = (c["bmax"] + 1.0) / c["bmin"]
    rung_bytes = 0
    for k in range(int(math.ceil(math.log(c["pmax"] / c["pmin"]) / math.log(g)))):
        f = f0 * g ** k
        n = int(math.floor(n_in / f))
        if min(c["bmax"], n, int(c["pmax"] / (f * tsamp))) >= c["bmin"]:
            rung_bytes += 4 * n_in + 4 * n
    return rung_bytes + 4 * stats["cells"] + 4 * plan.length * plan.num_widths + 12 * plan.length


def _drop_cache(fn):
    """fsync the file and drop it from the page cache, so the next read of it
    comes from the disk (POSIX_FADV_DONTNEED; best effort)."""
    fd = os.open(fn, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)


def bench_cfg5(args, torch, dist, world, rank, local, dev):
    """BASELINE configs[4] (cfg5): SIGPROC .tim DM trials of 2^23 samples @ 64 us
    searched from files to clustered peak lists, the rffa search and
    clustering stages (pipeline.py:177-215 with worker_pool.py:47-70) on the
    GPU worker pool:
    file read + H2D (8-bit files converted on the device) + deredden +
    normalise + 3 search ranges (example.yaml) + device peak detection, then
    the gathered peaks sorted by period and clustered in frequency
    (cluster1d, radius 0.2 / Tobs).
    Each rank searches its round-robin share of the node's file list
    (dispatch.search_files: DMIterator chunks of --batch files, the next chunk
    read into a bounded page-locked ring while the current one is on the
    device).  Two timed passes: `cold` after the files were fsync'ed and
    dropped from the page cache (the reads hit the disk; this is `value`),
    then `warm` (page cache)."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import inputs
    from riptide_amd.clustering import cluster_peaks
    from riptide_amd.dispatch import search_files
    from riptide_amd.reading import write_sigproc
    from riptide_amd.worker_pool import GpuWorkerPool
    c = inputs.CFG5
    root = os.environ.get("TMPDIR", "/tmp")
    files = args.files
    # ~8 MiB (8-bit) / 32 MiB (float32) per file; leave 20 % of the disk free
    free = shutil.disk_usage(root).free
    files = max(2 * args.batch, min(files, int(0.8 * free / world / (34 << 20))))
    if world > 1:
        # every rank must agree on the node's file list before any writes:
        # the smallest count over ranks (each measured the disk before writing)
        t = torch.tensor([files], dtype=torch.int64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        files = int(t.item())
    tmp = tempfile.mkdtemp(prefix=f"cfg5_r{rank}_", dir=root)
    # the node's file list (rank r writes the files it will search, k = r, r + world, ...)
    total = world * files
    fnames = [None] * total
    base = {}
    for k in range(rank, total, world):
        j = k % 64
        if j not in base:
            base[j] = inputs.cfg5_trial(j)
        data, hdr = base[j]
        fn = os.path.join(tmp, f"DM{hdr['refdm']:08.2f}_{k:05d}.tim")
        write_sigproc(fn, data, hdr)
        fnames[k] = fn
    base.clear()
    for k in range(rank, total, world):
        _drop_cache(fnames[k])
    if world > 1:      # every rank's paths (the others' entries are not read by this rank)
        parts = [None] * world
        dist.all_gather_object(parts, fnames[rank::world])
        for r in range(world):
            fnames[r::world] = parts[r]
    pool = GpuWorkerPool(c["dereddening"], c["ranges"], processes=args.batch, fmt="sigproc", batch=args.batch,
                         device=local)
    # warmup on a private copy (plans, device buffers, page-locked ring) so the
    # timed files stay cold
    wfn = os.path.join(tmp, "warmup.tim")
    d0, h0 = inputs.cfg5_trial(0)
    write_sigproc(wfn, d0, h0)
    pool.process_fname_list([wfn] * min(args.batch, 2))
    os.remove(wfn)
    res = {}
    for mode in ("cold", "warm"):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        peaks = search_files(fnames, pool, chunksize=args.batch)
        # Pipeline.search's sort + Pipeline.cluster_peaks (pipeline.py:186,
        # 192-215) on the gathered list, inside the timed region
        _, clusters = cluster_peaks(peaks, CFG5_CLUSTER_RADIUS, c["n"] * c["tsamp"])
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
            elapsed = rank_max(torch, dist, elapsed, dev)
        res[mode] = (elapsed, len(peaks), len(clusters))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        lst = os.path.join(tmp, "files.txt")
        with open(lst, "w") as f:
            f.write("\n".join(fnames))
        cpu = cpu_baselines("cfg5", extra=("--files-from", lst))
    if world > 1:
        dist.barrier()
    for k in range(rank, total, world):
        os.remove(fnames[k])
    shutil.rmtree(tmp, ignore_errors=True)
    if rank == 0:
        cold, warm = res["cold"], res["warm"]
        line = {
            "metric": "DM trials/sec files->peak clusters (cfg5 rffa search + clustering stages, 2^23 samples @ 64 us, 3 ranges)",
            "value": total / cold[0], "unit": "DM trials/s", "n_gpus": world, "steps": 1, "warmup": 1,
            "ms_per_step": cold[0] * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic SIGPROC files (tests/golden/inputs.py cfg5_trial k mod 64; 6 of 8 "
                                    "float32, 2 of 8 8-bit) written, fsync'ed and dropped from the page cache "
                                    "before the timed region (value: cold reads from disk)",
            "config": {"workload": "cfg5: rffa search stage on SIGPROC .tim files (example.yaml ranges short / "
                                   "medium / long, smin 6), dispatch.search_files, DMIterator chunks of --batch "
                                   "files with the next chunk prefetched",
                       "files_per_gpu": files, "chunk": args.batch,
                       "scratch_mfloats_per_buffer_trial": float(os.environ.get("RIPTIDE_AMD_SCRATCH_MFLOATS", "96")), "peaks_found": cold[1],
                       "clusters_found": cold[2], "clustering_radius_per_tobs": CFG5_CLUSTER_RADIUS,
                       "timed": "file read + H2D + deredden + normalise + 3 ranges' periodograms + device "
                                "peak detection + gather + sort by period + cluster1d (pipeline.py:177-215)",
                       "parallelism": f"dm-trials x{world} (independent, weak scaling)" + REHEARSAL},
            "cold": {"value": total / cold[0], "seconds": cold[0]},
            "warm": {"value": total / warm[0], "seconds": warm[0], "peaks_found": warm[1],
                     "clusters_found": warm[2]},
        }
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)


# example.yaml `clustering.radius` (units of 1 / Tobs; pipeline.py:200)
CFG5_CLUSTER_RADIUS = 0.2

CFG3 = dict(n=1 << 22, tsamp=256e-6, pmin=0.2, pmax=5.0, bmin=240, bmax=260, ducy_max=0.2,
            rmed_width=4.0, rmed_minpts=101, trials=1024)


# set by --one-gpu-rehearsal: every rank on cuda:0 over gloo (a code-path
# check of the multi-rank legs, not a measurement)
REHEARSAL = ""


def rank_max(torch, dist, x, dev):
    """Max of a float over the ranks (RCCL: a device tensor; gloo, the
    one-GPU rehearsal: a host tensor)."""
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def self_check(torch, dist, engine, plan, xbuf, snr, c, local, world, dev, ntrials):
    """After the timed region: EVERY trial of the last timed batch (their
    dereddened + normalised series are still in xbuf[0:ntrials]) through a
    plan with the library's default transform grouping (96 Mi floats per
    buffer, the schedule every GPU parity test runs) at batch 1 -- one trial
    per workgroup, so none of the benchmarked trial loop's later-trial paths
    (the next trial's fill overlapping this trial's stores, the zero-row
    rewrite) -- and True on every rank only if all ntrials S/N arrays are
    bit-identical to the benchmarked schedule's (snr[b])."""
    saved = {k: os.environ.pop(k, None) for k in ("RIPTIDE_AMD_SCRATCH_MFLOATS", "RIPTIDE_AMD_COSCHED",
                                                   "RIPTIDE_AMD_TRIALS_PER_WG")}
    try:
        ref = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                                ducy_max=c["ducy_max"], device=local)
    finally:
        for k, v in saved.items():
            if v is not None:
                os.environ[k] = v
    bad = []
    out = torch.empty((1, ref.length, ref.num_widths), dtype=torch.float32, device=dev)
    ws = torch.empty(ref.workspace_bytes(1), dtype=torch.uint8, device=dev)
    for b in range(ntrials):
        ref.run(xbuf[b:b + 1], out=out, workspace=ws, check=True)
        torch.cuda.synchronize()
        if not torch.equal(out[0], snr[b]):
            bad.append((b, int((out[0] != snr[b]).sum().item())))
    same = not bad
    if bad:
        print(f"bench self-check: S/N of trials differ from their batch-1 default-schedule runs "
              f"(trial, values): {bad}", file=sys.stderr, flush=True)
    del ref, out, ws
    if world > 1:
        same = rank_max(torch, dist, 0.0 if same else 1.0, dev) == 0.0
    return same


def cfg3_trials(torch, ks, n, tsamp, device):
    """BASELINE configs[2] trials, generated on the device: trial k is white
    noise from a generator seeded k, plus a slow red-noise ramp; every 64th
    trial carries a top-hat pulsar (period 0.2 + 4.8 * frac(0.618 k) s,
    amplitude 10-20)."""
    x = torch.empty((len(ks), n), dtype=torch.float32, device=device)
    g = torch.Generator(device=device)
    t = torch.arange(n, device=device, dtype=torch.float64) * tsamp
    ramp = (0.5 * torch.sin(2 * 3.141592653589793 * t / 700.0)).to(torch.float32)
    for i, k in enumerate(ks):
        g.manual_seed(k)
        torch.randn((n,), generator=g, device=device, dtype=torch.float32, out=x[i])
        x[i] += ramp
        if k % 64 == 0:
            period = 0.2 + 4.8 * ((0.6180339887 * k) % 1.0)
            amp = 10.0 + 10.0 * ((0.7548776662 * k) % 1.0)
            on = torch.remainder(t / period + 0.3, 1.0) < 0.02
            x[i] += on.to(torch.float32) * (amp / float(on.sum().item()) ** 0.5)
    return x


def bench_cfg3(args, torch, dist, world, rank, local, dev):
    """BASELINE configs[2] as configured: a job of 1024 DM trials x 2^22
    samples @ 256 us (P 0.2-5 s, bins 240-260, 10 widths), strong-sharded
    over the ranks (dispatch.shard(1024, rank, world), round-robin, no
    data-path collective), each rank's share resident in HBM.  One step = the
    whole job: deredden + normalise + periodogram of every trial, in device
    batches of --batch trials.  value = 1024 x steps / (max over ranks of the
    timed wall time)."""
    from riptide_amd import engine
    from riptide_amd.dispatch import shard
    c = CFG3
    ntr = args.trials or c["trials"]
    mine = shard(ntr, rank, world)
    B = min(args.batch, max(1, len(mine)))
    plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"], device=local)
    if os.environ.get("RIPTIDE_AMD_COSCHED") == "1":
        # two scratch banks only if they, the resident trials and the batch
        # buffers leave 10 % of the free HBM
        need = plan.workspace_bytes(B) + 4 * c["n"] * (len(mine) + 3 * B) + 4 * B * plan.length * plan.num_widths
        if need > 0.9 * torch.cuda.mem_get_info(dev)[0]:
            os.environ.pop("RIPTIDE_AMD_COSCHED")
            del plan
            plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"],
                                                     c["bmax"], ducy_max=c["ducy_max"], device=local)
    ws_samples = int(round(c["rmed_width"] / c["tsamp"]))
    X = cfg3_trials(torch, mine, c["n"], c["tsamp"], dev)
    xbuf = torch.empty((B, c["n"]), dtype=torch.float32, device=dev)
    dws = torch.empty(engine.deredden_workspace_bytes(c["n"], ws_samples, c["rmed_minpts"], B),
                      dtype=torch.uint8, device=dev)
    snr = torch.empty((B, plan.length, plan.num_widths), dtype=torch.float32, device=dev)
    pws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device=dev)

    def job():
        for b0 in range(0, len(mine), B):
            b1 = min(b0 + B, len(mine))
            engine.deredden_normalise(X[b0:b1], ws_samples, c["rmed_minpts"], out=xbuf[:b1 - b0], workspace=dws)
            plan.run(xbuf[:b1 - b0], out=snr[:b1 - b0], workspace=pws)

    for _ in range(args.warmup):
        job()
    torch.cuda.synchronize()
    plan.check()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    engine.profile_reset()
    engine.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    engine.profile_enable(False)
    plan.check()
    if world > 1:
        dist.barrier()
        elapsed = rank_max(torch, dist, elapsed, dev)
    cone = engine.profile_read(0)
    stats = plan.stats()
    # every trial of the last batch through the default-schedule plan at batch 1
    last = len(mine) - B * ((len(mine) - 1) // B)
    checked = None if args.no_self_check else self_check(torch, dist, engine, plan, xbuf, snr, c, local, world, dev,
                                                         last)
    if rank == 0:
        pmc, pmc_reason = pmc_traffic("cfg3")
        rf = roofline(engine, cone, stats, B, pmc, pmc_reason)
        rf["kernel_ms_per_trial"] = cone["ms"] / (args.steps * len(mine))
        nb = (len(mine) + B - 1) // B
        rf["timing"] = ("HIP events per cone launch" if cone["launches"] == stats["launches"] * args.steps * nb
                        else "HIP events around each batch's cone launch sequence (two streams)")
        fb = floor_bytes_per_trial(c, plan, stats)
        rf["floor_bytes_per_trial"] = fb
        rf["floor_frac"] = fb * ntr * args.steps / elapsed / 1e9 / HBM_PEAK_GBS
        rf["floor_basis"] = ("SURVEY.md §8(d): Σ_rungs(4N + 4n) + 4·Σ m·p + 4·L·W + 12·L per trial, x trials "
                             "/ wall time of the job / peak")
        line = {
            "metric": "DM trials/sec (node), 1024-trial job at 2^22 samples, P=0.2-5 s (BASELINE configs[2])",
            "value": ntr * args.steps / elapsed,
            "unit": "DM trials/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device-generated white noise + red-noise ramp, a top-hat pulsar in every 64th "
                    "trial; each rank's share resident in HBM)",
            "config": {
                "workload": "cfg3: 1024 DM trials x 2^22 samples @ 256 us, deredden(4 s, 101 pts) + normalise + "
                            "FFA periodogram P=0.2-5 s, bins 240-260, 10 widths; one step = the whole job",
                "trials_total": ntr, "trials_per_gpu": len(mine), "batch": B,
                "trial_periods": plan.length, "ffa_transforms": stats["transforms"],
                "cone_launches_per_batch": stats["launches"],
                "scratch_mfloats_per_buffer_trial": float(os.environ.get("RIPTIDE_AMD_SCRATCH_MFLOATS", "96")),
                "cosched_groups": os.environ.get("RIPTIDE_AMD_COSCHED") == "1",
                "parallelism": f"dm-trials x{world} (round-robin shard of one job, strong scaling)" + REHEARSAL,
            },
            "roofline": rf,
            "checked": checked,
            "checked_trials": None if checked is None else last,
            "check_basis": "every trial of the last timed batch == its batch-1 run through the default "
                           "96 M-float schedule, bit for bit",
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baselines("cfg3")
        print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0, help="DM trials per GPU per device batch "
                                                           "(default: 16 cfg2 / cfg5, 32 cfg3)")
    ap.add_argument("--workload", choices=("cfg2", "cfg3", "cfg5"), default="cfg2",
                    help="cfg2: headline periodogram throughput (device-resident, weak scaling); cfg3: the "
                         "1024-trial job of BASELINE configs[2] (strong scaling); cfg5: files -> peaks")
    ap.add_argument("--files", type=int, default=256, help="cfg5: SIGPROC files per GPU")
    ap.add_argument("--trials", type=int, default=0, help="cfg3: trials in the job (default 1024)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-self-check", action="store_true",
                    help="skip the post-timing S/N check against the default schedule (profiling runs: its "
                         "launches would be counted with the timed ones)")
    ap.add_argument("--one-gpu-rehearsal", action="store_true",
                    help="multi-rank code path check on a one-GPU box: every rank on cuda:0, gloo instead of "
                         "RCCL (not a measurement)")
    ap.add_argument("--overlap", type=int, default=0, choices=(0, 1),
                    help="cfg2: 1 = step k+1's deredden + normalise + downsampling ladder on a second stream "
                         "while step k's FFA passes run (two workspaces); 0 = one stream")
    args = ap.parse_args()
    if not args.batch:
        args.batch = 32 if args.workload == "cfg3" else 16

    # transform-group scratch per ping/pong buffer and trial (capi.cpp
    # scratch_budget_floats, tools/ab_sched.py): cfg2 at 1536 M floats puts
    # the whole plan in one group, 8 cone launches per step instead of 26 at
    # 384 M, 2.5 % faster (profiles/r03zd_sched_cfg2.jsonl), for 175 GB of
    # workspace at 16 trials (53 GB at 384 M), so only where it fits: one
    # workspace, one rank per GPU, and enough free HBM (checked below); cfg3
    # at 32 trials has few launches at 384 M already
    # Round 5: two 1024 M-float groups co-scheduled on two streams
    # (RIPTIDE_AMD_COSCHED=1: group g's merge-only passes run beside group
    # g - 1's S/N passes) for the same workspace as one 1536 M group: cfg2
    # cone 6.208-6.215 -> 6.160-6.169 ms per trial (profiles/r05zl_*.log)
    user_scratch = "RIPTIDE_AMD_SCRATCH_MFLOATS" in os.environ
    user_cosched = "RIPTIDE_AMD_COSCHED" in os.environ
    if args.workload in ("cfg2", "cfg3"):
        big = args.workload == "cfg2" and not args.overlap and not args.one_gpu_rehearsal
        if big and not user_scratch and not user_cosched:
            os.environ["RIPTIDE_AMD_COSCHED"] = "1"
            os.environ["RIPTIDE_AMD_SCRATCH_MFLOATS"] = "1024"
        # cfg3: its 384 M groups co-scheduled too, where the second bank fits
        # (bench_cfg3): cone 1.645-1.652 -> 1.637-1.639 ms per trial
        # (profiles/r05zn_ab_cosched_cfg3.log)
        if args.workload == "cfg3" and not user_cosched and not args.one_gpu_rehearsal:
            os.environ["RIPTIDE_AMD_COSCHED"] = "1"
        os.environ.setdefault("RIPTIDE_AMD_SCRATCH_MFLOATS", "1536" if big else "384")
    if args.workload == "cfg5" and not user_scratch:
        # cfg5's three range plans at 384 M floats per buffer and trial:
        # fewer transform groups and cone launches than the 96 M default,
        # 165.8 / 166.8 -> 185.4 DM trials/s (co-scheduling on top: 183.0;
        # profiles/r06i6_ab_cfg5_scratch.log), within HBM at batch 16
        os.environ["RIPTIDE_AMD_SCRATCH_MFLOATS"] = "384"
    import torch
    import torch.distributed as dist
    from riptide_amd import engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.one_gpu_rehearsal:
        global REHEARSAL
        local = 0
        REHEARSAL = " [one-GPU rehearsal: all ranks on cuda:0 over gloo, not a measurement]"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.one_gpu_rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    if args.workload in ("cfg3", "cfg5"):
        (bench_cfg3 if args.workload == "cfg3" else bench_cfg5)(args, torch, dist, world, rank, local, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    c = CFG
    plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"], device=local)
    B = args.batch
    if not user_scratch and os.environ["RIPTIDE_AMD_SCRATCH_MFLOATS"] != "384":
        # the one-group schedule only if its workspace + the step's buffers
        # leave 10 % of the free HBM; else the 384 M groups
        need = plan.workspace_bytes(B) + 4 * B * (plan.length * plan.num_widths + 3 * c["n"])
        if need > 0.9 * torch.cuda.mem_get_info(dev)[0]:
            os.environ["RIPTIDE_AMD_SCRATCH_MFLOATS"] = "384"
            if not user_cosched:
                os.environ.pop("RIPTIDE_AMD_COSCHED", None)
            del plan
            plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"],
                                                     c["bmax"], ducy_max=c["ducy_max"], device=local)
    ws_samples = int(round(c["rmed_width"] / c["tsamp"]))
    raw = synth_batch(torch, B, c["n"], c["tsamp"], 1000 + rank, dev)
    xbuf = torch.empty_like(raw)
    dws = torch.empty(engine.deredden_workspace_bytes(c["n"], ws_samples, c["rmed_minpts"], B),
                      dtype=torch.uint8, device=dev)
    snr = torch.empty((B, plan.length, plan.num_widths), dtype=torch.float32, device=dev)
    pws = [torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device=dev) for _ in range(1 + args.overlap)]
    s_main = torch.cuda.current_stream(dev)
    s_prep = torch.cuda.Stream(dev) if args.overlap else s_main
    ev_prep = [torch.cuda.Event() for _ in pws]
    ev_done = [torch.cuda.Event() for _ in pws]

    def run_steps(k_steps):
        # one step = deredden + normalise + ladder (prep) and the FFA passes +
        # S/N of one batch; with --overlap the prep of step k + 1 runs on
        # s_prep while step k's passes run on s_main (workspace k % 2; the
        # prep of step k + 2 waits for step k's passes to release it)
        for k in range(k_steps):
            w = k % len(pws)
            with torch.cuda.stream(s_prep):
                if args.overlap and k >= len(pws):
                    s_prep.wait_event(ev_done[w])
                engine.deredden_normalise(raw, ws_samples, c["rmed_minpts"], out=xbuf, workspace=dws, stream=s_prep)
                plan.ladder(xbuf, pws[w], stream=s_prep)
                ev_prep[w].record(s_prep)
            s_main.wait_event(ev_prep[w])
            plan.passes(snr, pws[w], stream=s_main)
            ev_done[w].record(s_main)
        s_main.wait_stream(s_prep)

    run_steps(args.warmup)
    torch.cuda.synchronize()
    plan.check()                  # device error flag of the warmup runs
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    engine.profile_reset()
    engine.profile_enable(True)
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    engine.profile_enable(False)
    plan.check()                  # every timed step: no unit refused (the flag is sticky)
    if world > 1:
        dist.barrier()
        elapsed = rank_max(torch, dist, elapsed, dev)
    cone = engine.profile_read(0)
    ladder = engine.profile_read(1)
    stats = plan.stats()
    checked = None if args.no_self_check else self_check(torch, dist, engine, plan, xbuf, snr, c, local, world, dev,
                                                         B)

    if rank == 0:
        pmc, pmc_reason = pmc_traffic()
        trials = world * B * args.steps
        rf = roofline(engine, cone, stats, B, pmc, pmc_reason)
        rf["kernel_ms_per_step"] = cone["ms"] / args.steps
        # one HIP-event record per cone launch, or one per launch sequence
        # when the plan's slot-width chains run on two streams (capi.cpp
        # run_cone_launches): then `achieved` is the sequence's algorithmic
        # bytes over its wall time, the two chains overlapping
        rf["profile_records_per_step"] = cone["launches"] / args.steps
        rf["timing"] = ("HIP events per cone launch" if cone["launches"] == stats["launches"] * args.steps
                        else "HIP events around each step's cone launch sequence (two streams)")
        rf["ladder_ms_per_step"] = ladder["ms"] / args.steps
        # progress against the implementation-independent floor (VERDICT r4:
        # the per-pass `frac` above rises if the schedule adds passes)
        fb = floor_bytes_per_trial(c, plan, stats)
        rf["floor_bytes_per_trial"] = fb
        rf["floor_frac"] = fb * trials / elapsed / 1e9 / HBM_PEAK_GBS
        rf["floor_basis"] = ("SURVEY.md §8(d): Σ_rungs(4N + 4n) + 4·Σ m·p + 4·L·W + 12·L per trial, x trials "
                             "/ wall time of the timed steps / peak")
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
                "cosched_groups": os.environ.get("RIPTIDE_AMD_COSCHED") == "1",
                "streams": "prep (deredden+normalise+ladder of step k+1) || FFA passes of step k" if args.overlap
                           else "one",
                "parallelism": f"dm-trials x{world} (independent, weak scaling)" + REHEARSAL,
            },
            "roofline": rf,
            "checked": checked,
            "checked_trials": None if checked is None else B,
            "check_basis": "every trial of the last timed batch == its batch-1 run through the default "
                           "96 M-float schedule, bit for bit",
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baselines("cfg2")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
