#!/usr/bin/env python3
"""Cold-read rate of this host's storage with 1, 2, 4 and 8 concurrent reader
processes over cfg5-shaped SIGPROC files: the input rate
an 8-GPU node's ranks would share in bench.py --workload cfg5 (each rank reads
its own round-robin share of the file list, dispatch.search_files).

CPU only.  Writes FILES files (bench.py's cfg5 mix: 6 of 8 float32 = 32 MiB,
2 of 8 8-bit = 8 MiB; header + 2^23 samples) under $TMPDIR, fsyncs them, and
for each reader count drops them from the page cache (POSIX_FADV_DONTNEED)
and times R processes reading disjoint round-robin shares with readinto()
into a reused buffer (bench.py's page-locked slots are filled the same way).

usage: python tools/read_rate.py [FILES] [OUT.jsonl] [DIR...]   (default DIR: $TMPDIR or /tmp)
"""
import json
import multiprocessing as mp
import os
import shutil
import sys
import tempfile
import time

NS = 1 << 23
CHUNK = 8 << 20


def _drop(fn):
    fd = os.open(fn, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)


def _fs_type(path):
    """(mount point, fs type, source) of the mount holding path (/proc/mounts,
    longest prefix): tmpfs / overlay on RAM make 'cold' reads page-cache reads."""
    best = ("", "?", "?")
    p = os.path.realpath(path)
    try:
        with open("/proc/mounts") as f:
            for line in f:
                src, mnt, typ = line.split()[:3]
                if (p == mnt or p.startswith(mnt.rstrip("/") + "/")) and len(mnt) > len(best[0]):
                    best = (mnt, typ, src)
    except OSError:
        pass
    return best


def _reader(fnames, start_evt, q):
    buf = bytearray(CHUNK)
    mv = memoryview(buf)
    start_evt.wait()
    t0 = time.perf_counter()
    nbytes = 0
    for fn in fnames:
        with open(fn, "rb", buffering=0) as f:
            while True:
                k = f.readinto(mv)
                if not k:
                    break
                nbytes += k
    q.put((nbytes, t0, time.perf_counter()))


def main():
    nfiles = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    out = sys.argv[2] if len(sys.argv) > 2 else ""
    roots = sys.argv[3:] or [os.environ.get("TMPDIR", "/tmp")]
    lines = [measure(nfiles, root) for root in roots]
    if out:
        with open(out, "w") as f:
            f.write("".join(json.dumps(x) + "\n" for x in lines))


def measure(nfiles, root):
    need = nfiles * (33 << 20)
    free = shutil.disk_usage(root).free
    if need > 0.8 * free:
        nfiles = max(8, int(0.8 * free / (33 << 20)))
    tmp = tempfile.mkdtemp(prefix="readrate_", dir=root)
    fnames = []
    try:
        blob32 = os.urandom(4 * NS)
        for k in range(nfiles):
            nb = NS if k % 8 in (3, 7) else 4 * NS          # 2 of 8 files 8-bit
            fn = os.path.join(tmp, f"f{k:04d}.tim")
            with open(fn, "wb") as f:
                f.write(b"\0" * 364)                          # a SIGPROC header's size
                f.write(memoryview(blob32)[:nb])
            fnames.append(fn)
        del blob32
        total = sum(os.path.getsize(f) for f in fnames)
        mnt, typ, src = _fs_type(root)
        res = {"files": nfiles, "bytes": total, "mean_file_mib": total / nfiles / 2**20, "root": root,
               "mount": mnt, "fs_type": typ, "fs_source": src,
               "cpus_affinity": len(os.sched_getaffinity(0)), "readers": {}}
        ctx = mp.get_context("spawn")
        for R in (1, 2, 4, 8):
            for fn in fnames:
                _drop(fn)
            ev = ctx.Event()
            q = ctx.Queue()
            ps = [ctx.Process(target=_reader, args=(fnames[r::R], ev, q)) for r in range(R)]
            for p in ps:
                p.start()
            time.sleep(0.5)                       # every reader started (spawn)
            ev.set()
            got = [q.get() for _ in ps]
            for p in ps:
                p.join()
            wall = max(g[2] for g in got) - min(g[1] for g in got)
            nb = sum(g[0] for g in got)
            res["readers"][str(R)] = {"GiB_per_s": nb / wall / 2**30, "files_per_s": nfiles / wall,
                                      "seconds": wall}
            print(f"{root} ({typ}) readers {R}: {nb / wall / 2**30:.2f} GiB/s, {nfiles / wall:.1f} files/s",
                  flush=True)
        print(json.dumps(res), flush=True)
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
