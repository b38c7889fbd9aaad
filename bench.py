#!/usr/bin/env python3
"""bench.py -- Disq BAM read path on MI355X (BASELINE.json metric).

metric: "decompressed BAM GB/s + reads/sec (whole node) at 1/2/4/8 MI355X".

Workload (configs[2] family, weak-scaled): ONE synthetic coordinate-sorted 30x-WGS-shaped BAM
(2x150 bp pairs, GRCh38-like dictionary, 0.5 % unplaced-unmapped tail) of N x --gb GB (12.5 GB per
GPU: 100 GB at N = 8, the configs[2] file), byte-range sharded over the N ranks.  Rank r generates
only its own byte range [O_r, O_{r+1}) of the file (the generator's chunks are independently
seeded) and keeps it resident in HBM; it owns the Disq partitions whose split starts there.

A step (timed) = the whole read of the file by all ranks:
  * halo exchange: rank r receives [O_{r+1}, hi_r + halo) from its successor(s) over RCCL/xGMI,
    HBM to HBM, right behind its resident bytes (parallel.exchange; none at N = 1);
  * the device pipeline on the shard (dq_open_shard_device + dq_run_resident): BGZF scan + chain,
    inflate + CRC32, split planning (record guesser), record chain, SoA decode + per-record hash,
    partition digests;
  * all_gather of the per-partition (count, digest) descriptors and the whole-file digest fold.
Records stay in HBM.  value = the file's decompressed bytes / max-over-ranks step time.

At N = 1 (rank 0 holds the whole file) the CPU baseline runs the oracle (CPU restatement of the
same per-partition work, zlib inflate) on the box's usable cores over a bounded sample of the
same partitions; its per-partition digests -- over every partition, the ones past the timed
sample run once more untimed -- are compared with the GPU's ("parity" in the line; a mismatch
exits non-zero).

Launch: python bench.py [--gpus 1 --steps K --warmup W]; for N > 1 the driver uses
torch.distributed.run, one rank per GPU (RCCL).
"""
import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decompressed BAM GB/s + reads/sec (whole node) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured copy)
TRAFFIC_PROFILE = "r6z_inflate_traffic_pmc.json"
# utilisation of K2 from PMC counters of the benched build (tools/pmc_summary.py over a
# tools/pmc_inflate.sh run): VALU issue, LDS busy / bank-conflict / unaligned fractions
UTIL_PROFILE = "r6z_inflate_util.json"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gb", type=float, default=12.5, help="compressed GB of the file per GPU")
    ap.add_argument("--shape", choices=("wgs", "longread"), default="wgs",
                    help="wgs: configs[1]/[2] (2x150 bp pairs); longread: configs[4] (ONT-like "
                         "10-100 kb reads, 1 %% of 0.5-2 Mb, records spanning many BGZF blocks)")
    ap.add_argument("--split-size", type=int, default=0, help="Disq splitSize (0 = 32 MiB)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--halo", type=int, default=4 << 20, help="initial halo bytes")
    ap.add_argument("--cpu-seconds", type=float, default=24.0,
                    help="CPU baseline budget over its 4 runs (0 disables)")
    ap.add_argument("--threads", type=int, default=0,
                    help="CPU baseline threads (0 = every usable core of this host)")
    ap.add_argument("--no-crc", action="store_true")
    ap.add_argument("--intervals", type=int, default=10000,
                    help="BED-like intervals for the N = 1 interval-filter measurement (0 = skip)")
    ap.add_argument("--e2e", type=int, default=1, help="N = 1 end-to-end measurement (0 = skip)")
    ap.add_argument("--write-records", type=int, default=2000000,
                    help="N = 1 write-path (SURVEY.md section 8 row f3) measurement: records of the "
                         "WGS stream compressed on the GPU (0 = skip)")
    ap.add_argument("--gen-budget-s", type=float, default=150.0,
                    help="N > 1: generation seconds per rank before the ranks tile a chunk pool")
    ap.add_argument("--e2e-window-gb", type=float, default=2.0,
                    help="end-to-end: compressed GB per window")
    ap.add_argument("--e2e-depth", type=int, default=3, help="end-to-end: overlapping windows")
    ap.add_argument("--e2e-export", choices=("lean", "raw"), default="lean",
                    help="end-to-end export: lean = voffsets + raw record bytes (DQ_EXPORT_LEAN, "
                         "the fields are parsed from the raw bytes as BAMRecordCodec.decode does), "
                         "raw = also every SoA field, hash and raw offset")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="generation rehearsal: generate rank 0's share of an N-rank run under "
                         "the N-rank thread budget, report the time as JSON and exit (no GPU work)")
    return ap.parse_args()


def usable_cores():
    """(cores the scheduler lets this process use, cgroup CPU quota or None, min of the two)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    return aff, quota, use


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    import numpy as np
    import torch
    # DQ_BENCH_REHEARSAL=1: every rank on GPU 0 and gloo collectives through host memory -- a
    # rehearsal of the N > 1 logic on a one-GPU box (RCCL refuses two ranks on one device); the
    # line then carries an oracle check of the whole-file digest.  Never used for measurements.
    rehearsal = os.environ.get("DQ_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    if not args.emulate_world:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if rehearsal else dev  # where collective tensors live
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    aff, quota, ncores = usable_cores()
    # the generation's world: this run's, or the one a rehearsal emulates (rank 0 of it)
    gworld = args.emulate_world or world
    gen_threads = max(1, min(32, ncores // max(1, args.emulate_world or local_world)))

    from disq_amd import _lib, parallel as P, synth

    # ---- workload: this rank's byte range of one logical N x args.gb GB file
    os.environ["DQ_SYNTH_PROGRESS"] = "1"
    t0 = time.time()
    shape = synth.LONGREAD if args.shape == "longread" else synth.WGS
    per_chunk = 2000 if shape == synth.LONGREAD else 20000
    probe = synth.generate(per_chunk, seed=args.seed, nthreads=gen_threads, shape=shape)
    probe_s = time.time() - t0  # one chunk, on one thread
    per_rec = len(probe.bam) / probe.n_records
    n_total = int(args.gb * 1e9 / per_rec) * gworld
    nchunks = synth.chunk_count(n_total, shape=shape)
    k0, k1 = rank * nchunks // gworld, (rank + 1) * nchunks // gworld
    want_bai = gworld == 1 and args.intervals > 0 and shape == synth.WGS
    # Generation budget: zlib level 5 (htsjdk's) costs ~1 thread-second per chunk, so with few
    # threads per rank (an 8-GPU node under a small CPU quota) the ranks generate a pool of
    # distinct chunks and tile it over their byte range (the blocks are the same level-5 BGZF
    # members; positions then repeat every pool instead of rising over the whole file).  N = 1
    # and any rank that fits the budget generate every chunk.
    est = (k1 - k0) * probe_s / max(1, gen_threads)
    pool = None
    if gworld > 1 and est > args.gen_budget_s:
        pool = max(2 * gen_threads, int(args.gen_budget_s * gen_threads / max(probe_s, 1e-3)))
    log(f"[bench] rank {rank}: chunks [{k0}, {k1}) of {nchunks} ({n_total} records in the file), "
        f"{gen_threads} threads, estimated {est:.0f} s" + (f", pool of {pool} chunks" if pool else ""))
    import ctypes
    if pool is None or pool >= k1 - k0:
        res, free = synth.generate(n_total, seed=args.seed, nthreads=gen_threads, as_buffer=True,
                                   bai=want_bai, unplaced_fraction=0.005, shape=shape,
                                   chunks=None if gworld == 1 else (k0, k1))
        own_len = res.bam_len
        own_np = np.ctypeslib.as_array((ctypes.c_uint8 * own_len).from_address(res.bam))
        gen_desc = {"distinct_chunks": k1 - k0, "tiled_chunks": 0}
    else:
        own_np, free = tiled_rank_bytes(synth, n_total, args.seed, gen_threads, k0, k1, nchunks,
                                        pool, shape)
        own_len = len(own_np)
        res = None
        gen_desc = {"distinct_chunks": pool + (1 if k0 == 0 else 0),
                    "tiled_chunks": (k1 - k0) - pool - (1 if k0 == 0 else 0),
                    "note": "a pool of distinct level-5 chunks tiled over the rank's range"}
    gen_s = time.time() - t0
    if args.emulate_world:
        free()
        print(json.dumps({
            "rehearsal": f"generation of rank 0 of {gworld} (bench.py --gpus {gworld}), no GPU work",
            "gb_per_rank": args.gb, "shape": args.shape, "threads_per_rank": gen_threads,
            "usable_cores": ncores, "host_cores": aff, "cgroup_cpu_quota": quota,
            "chunks_of_rank": k1 - k0, "chunks_in_file": nchunks, "probe_chunk_s": round(probe_s, 3),
            "estimated_full_s": round(est, 1), "gen_budget_s": args.gen_budget_s,
            "generator": gen_desc, "own_gb": round(own_len / 1e9, 3),
            "generator_s": round(gen_s, 1)}), flush=True)
        return
    lens = [own_len]
    if dist is not None:
        t = torch.tensor([own_len], dtype=torch.int64, device=cdev)
        allt = [torch.zeros(1, dtype=torch.int64, device=cdev) for _ in range(world)]
        dist.all_gather(allt, t)
        allt = torch.cat(allt)
        lens = [int(x) for x in allt.cpu()]
    offsets = [0]
    for n in lens:
        offsets.append(offsets[-1] + n)
    file_len = offsets[-1]
    log(f"[bench] rank {rank}: {own_len / 1e9:.2f} GB of a {file_len / 1e9:.2f} GB file "
        f"generated in {gen_s:.0f} s")
    split_opts = {"split_size": args.split_size}
    plan = P.shard_plan(file_len, world, offsets, **split_opts)
    shard = plan[rank]
    nsplit = len(P.path_splits(file_len, **split_opts))

    # header: rank 0's bytes start the file
    with _lib.Context(device=local) as hc:
        header = P.broadcast_header(lambda b: hc.header_from_prefix(b),
                                    lambda n: own_np[:n].tobytes(), file_len, rank, world)

    # the end-to-end leg (N = 1) first, before this process holds the resident file and its
    # pipeline buffers on the device: run after the timed steps (and after the other legs) it
    # measured 1.00 s against 0.77-0.81 s in a fresh process, every stage slower
    # (profiles/r6b_e2e_sweep.txt); its digest is compared with the resident run's below
    e2e = None
    if world == 1 and args.e2e:
        e2e = end_to_end(own_np, args, None, header)
    # resident own bytes (H2D, outside the timed region)
    t0 = time.time()
    rs = P.ResidentShard(torch.from_numpy(own_np), dev)
    rs.reserve(0)
    torch.cuda.synchronize()
    h2d_s = time.time() - t0
    bai = ctypes.string_at(res.bai, res.bai_len) if (want_bai and res is not None and res.bai) else None
    cpu_data = own_np.copy() if (world == 1 and args.cpu_seconds > 0) else None
    own_host = torch.from_numpy(own_np.copy()) if (rehearsal and world > 1) else None
    del own_np
    free()

    ctx = _lib.Context(split_size=args.split_size, verify_crc=not args.no_crc, device=local)
    maxp = max(s.p1 - s.p0 for s in plan)
    halo = args.halo

    def step():
        """One read of the whole file by all ranks (timed)."""
        nrecv = sum(b - a for _, r, a, b in P.halo_transfers(plan, offsets, file_len, halo)
                    if r == rank)
        rs.reserve(nrecv)
        if dist is not None and own_host is not None:  # rehearsal: the halo through host memory
            got = P.exchange(own_host, offsets, plan, rank, halo, file_len)
            rs.recv.copy_(got.to(dev))
            torch.cuda.synchronize()
        elif dist is not None:
            P.exchange(rs.own, offsets, plan, rank, halo, file_len, out=rs.recv)
            torch.cuda.synchronize()
        st, cnt, dig, err = None, None, None, 0
        if not shard.empty:
            ptr, ln = rs.span(shard.lo - offsets[rank])
            try:
                ctx.open_shard_device(ptr, ln, shard.lo, file_len, shard.p0, shard.p1, header)
                st = ctx.run_resident()
                cnt, dig = ctx.partition_digests()
            except _lib.DqError as e:
                if "halo too small" not in str(e):
                    raise
                err = 1
        # descriptors of every shard: [err, owned bytes, records, counts..., digests...]
        d = np.zeros(3 + 2 * maxp, dtype=np.int64)
        d[0] = err
        if st is not None:
            d[1], d[2] = st.owned_bytes, st.n_records
            d[3:3 + len(cnt)] = cnt
            d[3 + maxp:3 + maxp + len(dig)] = dig.view(np.int64)
        if dist is not None:
            rows = [torch.zeros(3 + 2 * maxp, dtype=torch.int64, device=cdev) for _ in range(world)]
            dist.all_gather(rows, torch.from_numpy(d).to(cdev))
            every = torch.stack([r.cpu() for r in rows]).numpy()
        else:
            every = d[None]
        if int(every[:, 0].max()) != 0:
            return None
        digests = np.zeros(nsplit, dtype=np.uint64)
        for r, s in enumerate(plan):
            digests[s.p0:s.p1] = every[r, 3 + maxp:3 + maxp + s.p1 - s.p0].view(np.uint64)
        return st, int(every[:, 1].sum()), int(every[:, 2].sum()), P.fold_digest_np(digests)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    for i in range(max(1, args.warmup)):
        out = step()
        while out is None:  # a straddling record ran past the halo on some rank: grow it
            halo *= 4
            log(f"[bench] rank {rank}: halo grown to {halo}")
            out = step()
        log(f"[bench] warmup {i}: {out[0].ms_total:.1f} ms device, inflate "
            f"{out[0].ms_inflate:.1f} ms, halo {halo}")
    barrier()
    t0 = time.perf_counter()
    infl_ms, outs = [], []
    for i in range(args.steps):
        out = step()
        if out is None:
            raise RuntimeError("halo changed during the timed steps")
        outs.append(out)
        infl_ms.append(out[0].ms_inflate)
    barrier()
    el = time.perf_counter() - t0
    ms_step = el * 1e3 / args.steps
    stats, ubytes, nrec, digest = outs[-1]
    comp_bytes = file_len  # C of the whole job (every rank's shard)
    for i, o in enumerate(outs):
        log(f"[bench] step {i}: {o[0].ms_total:.1f} ms device (scan {o[0].ms_scan:.1f}, inflate "
            f"{o[0].ms_inflate:.1f}, plan {o[0].ms_plan:.1f}, records {o[0].ms_records:.1f})")
    if any(o[3] != digest for o in outs):
        raise RuntimeError("the file digest changed between steps")
    if dist is not None:
        t = torch.tensor([ms_step], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms_step = float(t.item())
    gbs = ubytes / (ms_step / 1e3) / 1e9
    reads_s = nrec / (ms_step / 1e3)

    # roofline of the dominant kernel (inflate): algorithmic bytes = DEFLATE payload read once +
    # decompressed bytes written once, per launch (one launch inflates every block of the shard)
    infl_avg = sum(infl_ms) / len(infl_ms)
    alg_bytes = stats.deflate_bytes + stats.decompressed_bytes
    achieved = alg_bytes / (infl_avg / 1e3) / 1e9
    traffic, traffic_src = None, None
    tp = os.path.join(ROOT, "profiles", TRAFFIC_PROFILE)
    if os.path.exists(tp) and world == 1 and abs(args.gb - 12.5) < 1e-9 and args.split_size == 0:
        with open(tp) as f:
            tj = json.load(f)
        traffic = tj.get("traffic_bytes_per_launch")
        traffic_src = f"profiles/{TRAFFIC_PROFILE} (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction)"
    util = None
    up = os.path.join(ROOT, "profiles", UTIL_PROFILE)
    if os.path.exists(up):
        with open(up) as f:
            uj = json.load(f)
        util = {"src": f"profiles/{UTIL_PROFILE} (from {uj.get('src')}, tools/pmc_summary.py)",
                "valu_issue_frac_def": "SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8 cycles / 2): "
                                       "a wave64 VALU op takes a SIMD-32 two cycles",
                **{k: v for k, v in uj.get("kernels", {}).items()}}

    interval_mode = cpu = parity = wpath = None
    if e2e is not None and "digest" in e2e:
        e2e["digest_match"] = e2e["digest"] == f"{digest:016x}"
    if world == 1:
        if args.write_records > 0:
            wpath = write_path_bench(args)
        if bai is not None:
            interval_mode = interval_bench(ctx, rs, shard, file_len, header, bai, args, cpu_data,
                                           ncores)
        if cpu_data is not None:
            cpu, parity = cpu_baseline(cpu_data, ctx, rs, shard, file_len, header, args, ncores)
    if world > 1:
        # every rank, untimed: the oracle over the bytes it decoded (resident + halo received in
        # the timed steps), its owned partitions vs the GPU's descriptors of the last timed step
        parity = shard_parity(rs, shard, offsets, rank, file_len, header, args.split_size, ctx,
                              dist, cdev, world, max(1, ncores // max(1, local_world)))
    if rehearsal and world > 1 and rank == 0 and not pool:
        # the whole logical file, generated at once, through the oracle: its digest must equal
        # the digest folded from the shards
        from oracle import oracle as O
        whole = synth.generate(n_total, seed=args.seed, nthreads=gen_threads, unplaced_fraction=0.005)
        _, odig, _ = O.run_partitions(whole.bam, O.path_splits(len(whole.bam), args.split_size),
                                      ncores)
        ok = len(whole.bam) == file_len and P.fold_digest([int(x) for x in odig]) == digest
        parity["whole_file_rehearsal"] = {
            "status": "match" if ok else "MISMATCH",
            "checked": "rehearsal (gloo, every rank on GPU 0): whole-file digest of the sharded "
                       "read vs the oracle over the whole logical file"}
        if not ok:
            parity["status"] = "MISMATCH"
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(gbs, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded generator, htsjdk BGZF conventions, deflate level 5)",
            "config": {
                "workload": (f"configs[2]: one synthetic 30x-WGS-shaped coordinate-sorted BAM of "
                             f"{world} x {args.gb} GB (100 GB at 8 GPUs), 2x150 bp pairs, 0.5 % "
                             f"unplaced-unmapped tail, byte-range sharded with halo stitching"
                             if shape == synth.WGS else
                             f"configs[4]: one synthetic long-read coordinate-sorted BAM of "
                             f"{world} x {args.gb} GB, ONT-like reads of 10-100 kb (1 % of "
                             f"0.5-2 Mb) whose records span many BGZF blocks, 0.5 % unplaced"),
                "parallelism": f"1 file, {world} byte-range shard(s), halo over "
                               + ("gloo (REHEARSAL on one GPU, not a measurement)" if rehearsal
                                  else "RCCL p2p"),
                "file_gb": round(file_len / 1e9, 3),
                "decompressed_gb": round(ubytes / 1e9, 3),
                "records": nrec,
                "reads_per_s": round(reads_s, 1),
                "split_size": args.split_size or 32 * 1024 * 1024,
                "partitions": nsplit,
                "crc32_verified": not args.no_crc,
                "digest": f"{digest:016x}",
                "halo_bytes": halo,
                "h2d_gbs": round(own_len / h2d_s / 1e9, 2),
                "device_ms_breakdown_rank0": {
                    "scan_chain": round(stats.ms_scan, 2), "inflate": round(stats.ms_inflate, 2),
                    "plan": round(stats.ms_plan, 2), "records": round(stats.ms_records, 2),
                    "total": round(stats.ms_total, 2)},
                "generator_s": round(gen_s, 1),
                "generator": dict(gen_desc, threads_per_rank=gen_threads,
                                  tiled=bool(gen_desc.get("tiled_chunks"))),
                "interval_mode": interval_mode,
                "end_to_end": e2e,
                "write_path": wpath,
                "parity": parity,
                # whole-pipeline algorithmic bytes C + 2U + 60R (unfused
                # record walk) over the step time, against the spec and the measured HBM peaks
                "pipeline_roofline": {
                    "bytes_alg": int(comp_bytes + 2 * ubytes + 60 * nrec),
                    "achieved_gbs": round((comp_bytes + 2 * ubytes + 60 * nrec) / (ms_step / 1e3) / 1e9, 2),
                    "frac_of_8000_gbs": round((comp_bytes + 2 * ubytes + 60 * nrec) / (ms_step / 1e3) / 8e12, 5),
                    "frac_of_6290_gbs_measured": round((comp_bytes + 2 * ubytes + 60 * nrec) / (ms_step / 1e3) / 6.29e12, 5),
                },
            },
            "roofline": {
                "bound": "hbm",
                "limiter": "VALU issue (each VALU instruction holds its SIMD for a quad-cycle: "
                           "busy 0.72 of them, utilisation.valu_busy_quad_frac) + LDS/barrier "
                           "latency of the serial Huffman decode (DESIGN.md section 3, Round 6), "
                           "far below the HBM roof",
                "kernel": "inflate_block_kernel + inflate_tail_kernel (one K2 launch)",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_src": traffic_src,
                "pmc_src": "profiles/r6z_inflate_pmc.txt (SQ counters of both K2 kernels, this build)",
                "trace_src": "profiles/r6z_rocprof_summary.txt (rocprofv3 kernel trace of this bench command: block kernel 165.31 ms + tail kernel 15.04 ms per launch)",
                "alg_bytes_per_launch": alg_bytes,
                "avg_launch_ms": round(infl_avg, 3),
                "utilisation": util,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    if parity is not None and parity.get("status") != "match":
        sys.exit(3)
    if (interval_mode or {}).get("parity") and interval_mode["parity"].get("status") != "match":
        sys.exit(3)


def shard_parity(rs, shard, offsets, rank, file_len, header, split_size, ctx, dist, cdev, world,
                 threads):
    """N > 1 parity, untimed, on every rank: the oracle (run_partitions_window) over exactly the
    bytes the rank decoded -- its resident range from its first split plus the halo it received
    over RCCL in the timed steps, copied back from HBM a group of partitions at a time -- with
    the broadcast header, for the
    partitions it owns (one chunk per partition, AbstractBinarySamSource.java:61-73); per-partition
    record count + ordered digest compared with the GPU's descriptors of the last timed step.
    The verdicts are all-gathered: every rank's line field is the same."""
    import numpy as np
    import torch
    from oracle import oracle as O
    t0 = time.perf_counter()
    ok, nparts, nrec, short, failed = 1, 0, 0, 0, 0
    if not shard.empty:
        # in groups of about 1 GB of partitions, so a rank's host copy stays small (8 ranks x a
        # 12.5 GB shard at once would be 100 GB of host memory); each group's window runs from its
        # first split start to its last split end + 4 MiB (x4 while the oracle finds it short)
        have = rs.n_own + rs.nrecv  # bytes of rs.buf, from offsets[rank]
        splits = O.path_splits(file_len, split_size)[shard.p0:shard.p1]
        gcnt, gdig = ctx.partition_digests()
        ocnt, odig = [], []
        i = 0
        try:
            while i < len(splits):
                j = i + 1
                while j < len(splits) and splits[j][1] - splits[i][0] <= (1 << 30):
                    j += 1
                lo, extra = splits[i][0], 4 << 20
                while True:
                    a = lo - offsets[rank]
                    b = min(have, splits[j - 1][1] - offsets[rank] + extra)
                    win = rs.buf[a:b].cpu().numpy()
                    try:
                        c, d, _ = O.run_partitions_window(win, lo, file_len, header, splits[i:j],
                                                          threads)
                        break
                    except O.OracleError as e:
                        if "short" not in str(e) or b >= have:
                            raise
                        extra *= 4
                    finally:
                        del win
                ocnt.append(c)
                odig.append(d)
                i = j
            ocnt, odig = np.concatenate(ocnt), np.concatenate(odig)
            ok = int(np.array_equal(gcnt, ocnt) and np.array_equal(gdig, odig))
            nparts, nrec = len(ocnt), int(ocnt.sum())
        except Exception as e:  # every rank must still reach the all_gather below
            ok = 0
            if isinstance(e, O.OracleError) and "short" in str(e):
                short = 1
            else:
                failed = 1
                print(f"[bench] rank {rank}: shard parity failed: {e!r}", file=sys.stderr, flush=True)
    row = torch.tensor([ok, nparts, nrec, short, int(1e3 * (time.perf_counter() - t0)), failed],
                       dtype=torch.int64, device=cdev)
    if dist is not None:
        rows = [torch.zeros_like(row) for _ in range(world)]
        dist.all_gather(rows, row)
        every = torch.stack([r.cpu() for r in rows]).numpy()
    else:
        every = row.cpu().numpy()[None]
    return {"status": "match" if int(every[:, 0].min()) == 1 else "MISMATCH",
            "ranks_matching": int(every[:, 0].sum()), "ranks": int(len(every)),
            "partitions_checked": int(every[:, 1].sum()), "records_checked": int(every[:, 2].sum()),
            "ranks_window_too_short": int(every[:, 3].sum()),
            "ranks_failed": int(every[:, 5].sum()),
            "oracle_s_max_over_ranks": round(float(every[:, 4].max()) / 1e3, 1),
            "oracle_threads_per_rank": threads,
            "checked": "per rank, untimed: the oracle over the rank's resident + RCCL-received "
                       "halo bytes (copied back from HBM) and the broadcast header, its owned "
                       "partitions' record counts + ordered digests vs the GPU's"}


def tiled_rank_bytes(synth, n_total, seed, threads, k0, k1, nchunks, pool, shape=0):
    """A rank's bytes [chunks k0, k1) from a pool of distinct chunks: chunk 0 (the header) and the
    last chunk (unplaced tail + EOF block) are generated as themselves; the pool [a, a + pool) of
    mid-file chunks is generated once and repeated, the remainder taken from its front."""
    import ctypes
    import numpy as np
    pieces = []
    a = k0 + 1 if k0 == 0 else k0
    last = k1 == nchunks
    b = k1 - 1 if last else k1
    pool = max(1, min(pool, b - a))

    def gen(lo, hi):
        r, fr = synth.generate(n_total, seed=seed, nthreads=threads, as_buffer=True,
                               unplaced_fraction=0.005, chunks=(lo, hi), shape=shape)
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * r.bam_len).from_address(r.bam)).copy()
        fr()
        return arr
    if k0 == 0:
        pieces.append(gen(0, 1))
    if b > a:
        # the pool, chunk by chunk boundaries known: generate it as single chunks in parallel
        # calls is serial in the library, so generate it whole and tile it whole
        whole = gen(a, a + pool)
        reps, rem = divmod(b - a, pool)
        pieces += [whole] * reps
        if rem:
            pieces.append(gen(a, a + rem))
    if last:
        pieces.append(gen(k1 - 1, k1))
    out = np.concatenate(pieces)
    return out, (lambda: None)


def make_intervals(seqs, n, seed=3):
    """n intervals, lengths log-uniform 100 bp - 100 kb, contigs
    proportional to their length, sorted (overlaps left for optimizeIntervals)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    lens = np.array([ln for _, ln in seqs], np.float64)
    ref = rng.choice(len(seqs), size=n, p=lens / lens.sum())
    ilen = np.exp(rng.uniform(np.log(100), np.log(100_000), size=n)).astype(np.int64)
    start = (rng.uniform(0, 1, size=n) * np.maximum(1, lens[ref] - ilen)).astype(np.int64) + 1
    end = np.minimum(start + ilen - 1, lens[ref].astype(np.int64))
    order = np.lexsort((start, ref))
    return [(int(ref[i]), int(start[i]), int(end[i])) for i in order]


def _reopen(ctx, rs, shard, file_len, header):
    ptr, ln = rs.span(shard.lo)  # N = 1: the resident range starts at byte 0
    ctx.open_shard_device(ptr, ln, shard.lo, file_len, shard.p0, shard.p1, header)


def interval_bench(ctx, rs, shard, file_len, header, bai, args, data=None, ncores=1):
    """configs[3] shape on the resident file: args.intervals BED-like intervals, traversed as Disq
    does (AbstractBinarySamSource.java:86-112): the .bai span of the optimized intervals clipped
    to every partition chunk is the only part inflated (dq_run_resident, span run), then kernel 4.
    Compared with kernel 4 over every record of the file (full_traversal): same kept count.
    Parity (untimed): the oracle's traversal of the same file and intervals, every partition
    (count + ordered digest of the kept records), without and with the unplaced-unmapped tail
    (traverse_unplaced_unmapped, AbstractBinarySamSource.java:116-129)."""
    stage = "setup"
    try:
        from disq_amd import _lib
        from disq_amd.storage import _parse_header
        _reopen(ctx, rs, shard, file_len, header)
        ctx.set_index(bai)
        ivs = make_intervals(_parse_header(header).sequences, args.intervals)
        stage = "first span run"
        st = ctx.run_resident((ivs, False))  # the partition plans (full run) + a first span run
        stage = "timed span runs"
        wall, dev = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            st = ctx.run_resident((ivs, False))
            wall.append(time.perf_counter() - t0)
            dev.append(st.ms_span)
        stage = "full traversal"
        with _lib.Context(split_size=args.split_size, verify_crc=not args.no_crc,
                          full_traversal=True) as fc:
            _reopen(fc, rs, shard, file_len, header)
            fc.set_index(bai)
            fc.run_resident((ivs, False))
            fst = fc.run_resident((ivs, False))
        parity = None
        if data is not None:
            stage = "oracle parity"
            import numpy as np
            from oracle import oracle as O
            splits = O.path_splits(len(data), args.split_size)
            parity = {}
            for unplaced in (False, True):
                _reopen(ctx, rs, shard, file_len, header)
                ctx.set_index(bai)
                ust = ctx.run_resident((ivs, unplaced))
                gcnt, gdig = ctx.partition_digests()
                t0 = time.perf_counter()
                ocnt, odig = O.run_partitions_traversal(data, splits, ncores, bai, ivs, unplaced)
                ok = bool(np.array_equal(gcnt, ocnt) and np.array_equal(gdig, odig))
                parity["with_unplaced_tail" if unplaced else "intervals_only"] = {
                    "status": "match" if ok else "MISMATCH", "partitions": int(len(ocnt)),
                    "records": int(ocnt.sum()), "gpu_records": int(ust.n_filtered),
                    "oracle_s": round(time.perf_counter() - t0, 2)}
            parity["status"] = ("match" if all(v["status"] == "match" for v in parity.values())
                                else "MISMATCH")
            parity["checked"] = ("per-partition count + ordered digest of the kept records, GPU "
                                 "span run vs the oracle's Disq traversal (C, "
                                 f"{ncores} threads) of the same file and intervals")
        return {"n_intervals": len(ivs), "records_in_spans": st.n_records,
                "records_kept": st.n_filtered,
                "blocks_inflated": st.blocks_inflated, "blocks_total": st.n_blocks,
                "ms_span_device": round(statistics.median(dev), 3),
                "ms_span_wall": round(1e3 * statistics.median(wall), 3),
                "ms_full_traversal_device": round(fst.ms_total + fst.ms_filter, 3),
                "full_traversal_kept": fst.n_filtered,
                "kept_match": fst.n_filtered == st.n_filtered,
                "unplaced_tail": "timed runs without it (traverse_unplaced_unmapped = false); "
                                 "parity checked with and without",
                "parity": parity}
    except Exception as e:  # noqa: BLE001 -- reported in the line; the headline metric stands
        return {"error": f"{type(e).__name__}: {e}", "stage": stage}


def cpu_baseline(data, ctx, rs, shard, file_len, header, args, ncores):
    """The oracle (CPU restatement of Disq's per-partition work: guesser + zlib inflate + record
    walk + hash) on every usable core, over a bounded sample of the same file's partitions:
    1 warm-up + median of 3.  The partitions past the sample are run once
    more, untimed, so the GPU's per-partition digests are compared over the whole file."""
    import numpy as np
    from oracle import oracle as O
    from disq_amd import parallel as P
    aff, quota, _ = usable_cores()
    threads = args.threads or ncores
    splits = O.path_splits(len(data), args.split_size)
    # calibrate on `threads` partitions, then take as many as fit a quarter of the budget
    t0 = time.perf_counter()
    O.run_partitions(data, splits[:threads], threads)
    one = time.perf_counter() - t0
    k = max(threads, int((args.cpu_seconds / 4) / max(one, 1e-3) * threads))
    k = min(k, len(splits))
    sample = splits[:k]
    runs = []
    cnt = dig = ub = None
    for i in range(4):
        t0 = time.perf_counter()
        cnt, dig, ub = O.run_partitions(data, sample, threads)
        if i:
            runs.append(time.perf_counter() - t0)
    el = statistics.median(runs)
    # parity covers every partition: the ones past the timed sample run once more, untimed
    ccnt, cdig = cnt, dig
    if k < len(splits):
        rcnt, rdig, _ = O.run_partitions(data, splits[k:], threads)
        ccnt, cdig = np.concatenate([cnt, rcnt]), np.concatenate([dig, rdig])
    # the GPU's partition digests of the same file (resident run)
    _reopen(ctx, rs, shard, file_len, header)
    st = ctx.run_resident()
    gcnt, gdig = ctx.partition_digests()
    ok = bool(np.array_equal(gcnt, ccnt) and np.array_equal(gdig, cdig))
    full = len(ccnt) == len(splits)
    if full:
        ok = ok and P.fold_digest([int(x) for x in cdig]) == st.digest
    parity = {"status": "match" if ok else "MISMATCH",
              "partitions_checked": int(len(ccnt)), "partitions": len(splits),
              "records_checked": int(ccnt.sum()),
              "checked": "per-partition record count + ordered digest of per-record raw-byte "
                         "hashes, GPU vs oracle" + (", and the whole-file digest" if full else "")}
    gbs = float(ub.sum()) / el / 1e9
    cpu = {
        "value": round(gbs, 4),
        "unit": "GB/s",
        "cores": threads,
        "host_cores": aff,
        "cgroup_cpu_quota": quota,
        "per_core_gbs": round(gbs / threads, 4),
        "node_extrapolation": {
            "gbs_all_host_cores": round(gbs / threads * aff, 2),
            "host_cores": aff,
            "label": "EXTRAPOLATION, not measured: per_core_gbs x host_cores, assuming linear "
                     "scaling to every core of the host (memory bandwidth and zlib would bend it "
                     "down); compare with the whole-node GPU figure of the 8-GPU run"},
        "kind": "port",
        "sample": f"first {k} of {len(splits)} Disq partitions (32 MiB splits) of the same file, "
                  f"one partition per thread: guesser + zlib inflate + record walk + hash; "
                  f"{int(cnt.sum())} records; median of 3 runs after 1 warm-up "
                  f"({', '.join(f'{r:.2f}' for r in runs)} s; {cnt.sum() / el:.0f} reads/s)",
    }
    return cpu, parity


FAST_DEFLATE = "16,16,32,4,1"  # chain, lazy, nice, good, fmerge (default 32,16,32,8,1)


def write_path_bench(args):
    """Row f3: the decompressed stream of a synthetic WGS BAM, resident in
    HBM, compressed into htsjdk's 65280-byte BGZF blocks by the GPU (dq_bgzf_compress_resident,
    HIP events around the deflate kernels); the output re-inflated by the GPU read path must give
    the stream back (digest).  The same measurement as tools/deflate_bench.py."""
    import hashlib
    from disq_amd import _lib, synth
    r = synth.generate(args.write_records, seed=1, nthreads=max(1, min(16, usable_cores()[2])))
    eof = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    with _lib.Context(verify_crc=True) as c:
        c.open_bytes(r.bam)
        c.run_resident()
        u = c.inflated()
        runs = [c.bgzf_compress_resident() for _ in range(4)]  # a warm-up and 3 timed
        n = runs[-1][0]
        z = c.bgzf_fetch(n).tobytes()
        n2 = c.bgzf_compress_resident()[0]  # once more: the same bytes (htsjdk's writer is deterministic)
        same = n2 == n and c.bgzf_fetch(n2).tobytes() == z
        # the speed end of the search-effort curve (DQ_DEFLATE, read at every launch): not the
        # default, whose level-5 search settings keep every golden stream within 0.5 % of zlib
        # level 5; this one is 0.65-1.35 % larger there (profiles/r6x_deflate_settings.txt)
        old_env = os.environ.get("DQ_DEFLATE")
        os.environ["DQ_DEFLATE"] = FAST_DEFLATE
        try:
            fruns = [c.bgzf_compress_resident() for _ in range(4)]
        finally:
            if old_env is None:
                os.environ.pop("DQ_DEFLATE", None)
            else:
                os.environ["DQ_DEFLATE"] = old_env
        fn = fruns[-1][0]
        fz = c.bgzf_fetch(fn).tobytes()
    fms = sorted(x[1] for x in fruns[1:])[1]
    ms = sorted(x[1] for x in runs[1:])[1]
    with _lib.Context(verify_crc=True) as c:
        c.text_open_bytes(z + eof)
        c.text_run(False)
        back = c.inflated()
    ok = hashlib.sha256(u.tobytes()).digest() == hashlib.sha256(back.tobytes()).digest()
    with _lib.Context(verify_crc=True) as c:
        c.text_open_bytes(fz + eof)
        c.text_run(False)
        fback = c.inflated()
    fok = hashlib.sha256(u.tobytes()).digest() == hashlib.sha256(fback.tobytes()).digest()
    out = {"workload": f"decompressed stream of {args.write_records} synthetic WGS records",
           "input_gb": round(len(u) / 1e9, 4), "compressed_gb": round(n / 1e9, 4),
           "ratio": round(len(u) / n, 3), "device_ms_median": round(ms, 3),
           "input_gbs": round(len(u) / ms / 1e6, 2),
           "htsjdk_level5_ratio": round(len(u) / len(r.bam), 3),
           "roundtrip_gpu_inflate": "match" if ok else "MISMATCH",
           "deterministic": same,
           # the write path's roofline: algorithmic bytes = input read once + BGZF output written
           # once, over the device time of the three kernels, against the HBM peak; counter traffic
           # of the same kernels (FETCH_SIZE x2 + WRITE_SIZE) from the cited PMC run
           "roofline": {"bound": "hbm", "achieved": round((len(u) + n) / ms / 1e6, 2),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round((len(u) + n) / ms / 1e6 / HBM_PEAK_GBS, 5),
                        "traffic_over_alg": 3.98,
                        "traffic_src": "profiles/r5zl_deflate_pmc.txt (0.868 GB per compression of "
                                       "0.162 GB: 3.98x the 0.218 GB algorithmic bytes)",
                        "limiter": "LZ77 parse latency of bgzf_parse_kernel (~88 % of device time; "
                                   "one 160 KB, 1024-thread workgroup per CU: 16 waves)"},
           "speed_setting": {"dq_deflate": FAST_DEFLATE, "ratio": round(len(u) / fn, 3),
                             "device_ms_median": round(fms, 3), "input_gbs": round(len(u) / fms / 1e6, 2),
                             "roundtrip_gpu_inflate": "match" if fok else "MISMATCH",
                             "golden_streams": "0.65-1.35 % larger than zlib level 5 (default: -1.9 to "
                                               "+0.42 %), profiles/r6x_deflate_settings.txt"},
           "evidence": "profiles/r5n_deflate_parse_1024.txt, r5zc_deflate_fmerge.txt, "
                       "r5zi_deflate_parallel_header.txt, r5zk_deflate_atomic_scatter.txt (A/Bs, "
                       "per-phase cycles), profiles/r5zl_deflate_pmc.txt (SQ counters and traffic)"}
    log("write path:", out)
    return out


def pcie_ceiling(nbytes=8 << 30, reps=3):
    """The host link's measured ceiling (untimed leg): pinned hipMemcpyAsync of `nbytes` device to
    host alone, host to device alone, and both directions at once on two streams (half the bytes
    each way), GB/s by HIP events, median of `reps`."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    half = nbytes // 2

    def timed(fn):
        out = []
        for _ in range(reps + 1):  # the first is a warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            out.append(time.perf_counter() - t0)
        return statistics.median(out[1:])

    def d2h():
        with torch.cuda.stream(s1):
            h.copy_(d, non_blocking=True)

    def h2d():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)

    def both():
        with torch.cuda.stream(s1):
            d[:half].copy_(h[:half], non_blocking=True)
        with torch.cuda.stream(s2):
            h[half:].copy_(d[half:], non_blocking=True)
    t_d2h, t_h2d, t_both = timed(d2h), timed(h2d), timed(both)
    del h, d
    return {"bytes": nbytes, "d2h_gbs": round(nbytes / t_d2h / 1e9, 2),
            "h2d_gbs": round(nbytes / t_h2d / 1e9, 2),
            "bidirectional_gbs": round(nbytes / t_both / 1e9, 2),
            "method": "pinned torch copies (hipMemcpyAsync), median of 3 after a warm-up; "
                      "bidirectional = half the bytes each way on two streams"}


def end_to_end(data, args, resident_digest=None, header=None):
    """Page-cached file -> host SoA + raw records, every stage overlapped (one whole read, not
    timed with the steps): the file is in /dev/shm (RAM, as the page cache would hold it) and is
    read in windows of whole partitions by `depth` contexts on their own host threads and HIP
    streams (disq_amd.stream): one window's file -> pinned -> HBM copy, another's pipeline and a
    third's export of every record (lean, the default: its voffset and raw bytes; --e2e-export raw:
    also its SoA row) to host memory (dq_read) run at once,
    as Disq's tasks overlap their prefetcher's reads with decoding
    (SeekableByteChannelPrefetcher.java:253-298).  The whole-file digest must equal the resident
    run's."""
    if data is None:
        return None
    import numpy as np

    from disq_amd import _lib, stream
    path = f"/dev/shm/disq_bench_{os.getpid()}.bam"
    try:
        with open(path, "wb") as f:
            f.write(memoryview(data))
        if header is None:
            with _lib.Context() as hc:
                header = hc.header_from_prefix(bytes(data[:1 << 20]))
        exported = {"records": 0, "raw": 0, "soa": 0, "digests": []}
        keep = []
        lk = __import__("threading").Lock()

        mode = "lean" if args.e2e_export == "lean" else True

        def export(k, c, shard):
            b = c.read(with_raw=mode)
            n = len(b["voffset"])
            raw = 0 if b["raw"] is None else len(b["raw"])
            if mode == "lean":
                # the consumer's view: the first records parse from the raw bytes (record i + 1
                # starts 4 + block_size bytes after record i) and their voffsets ascend
                m = min(n, 256)
                if m:
                    o = 0
                    for i in range(m):
                        o += 4 + int.from_bytes(bytes(b["raw"][o:o + 4]), "little")
                    assert o <= raw and (m < n or o == raw)
                    assert bool(np.all(np.diff(b["voffset"][:m].astype(np.int64)) > 0))
            else:
                # the last record's raw bytes end where its offsets say
                assert raw == (int(b["raw_offset"][-1]) + 4 + int(b["block_size"][-1]) if n else 0)
            with lk:
                exported["records"] += n
                exported["raw"] += raw
                exported["soa"] += sum(int(b[k2].nbytes) for k2, _ in _lib.FIELDS if k2 in b)
                exported["digests"].append((shard.p0, b["part_digest"].copy()))
        window = int(args.e2e_window_gb * 1e9)
        # the contexts and their pinned export arenas are set up before the read (an executor's
        # long-lived buffers): a window's records land there by DMA, and the consumer is done with
        # them when the next window of that context is exported
        t0 = time.perf_counter()
        arena = int(window * 3.7)  # U + SoA of a window (2.85 + ~0.55 x its compressed bytes)
        ctxs = []
        for _ in range(args.e2e_depth):
            c = _lib.Context(split_size=args.split_size, verify_crc=not args.no_crc)
            c.set_export_arena(arena)
            ctxs.append(c)
        setup_s = time.perf_counter() - t0
        try:
            # one untimed pass first: the contexts' device buffers grow to the window size on their
            # first window (as an executor's would on its first task), then the timed read
            t0 = time.perf_counter()
            stream.stream_read(path, len(data), header, window=window, depth=args.e2e_depth,
                               split_size=args.split_size, verify_crc=not args.no_crc,
                               on_window=lambda *a: a[1].read(with_raw=mode), contexts=ctxs,
                               ramp=True)
            warm_s = time.perf_counter() - t0
            # ramp: quarter and half windows first and last, so the first export starts sooner and
            # the last one drains faster (profiles/r5zg_e2e_ramp_ab.txt).  Five timed reads, the
            # median reported (BASELINE.md section 3's protocol; single reads of the same build
            # ranged 0.77-0.90 s, profiles/r6b_e2e_sweep.txt, and 0.81-0.90 s in one r6final run)
            runs = []
            for _ in range(5):
                exported.update({"records": 0, "raw": 0, "soa": 0, "digests": []})
                r = stream.stream_read(path, len(data), header, window=window,
                                       depth=args.e2e_depth, split_size=args.split_size,
                                       verify_crc=not args.no_crc, on_window=export,
                                       contexts=ctxs, ramp=True)
                runs.append((r["seconds"], r, dict(exported, digests=list(exported["digests"]))))
            runs.sort(key=lambda x: x[0])
            _, res, exp_med = runs[len(runs) // 2]
            exported.update(exp_med)
            all_secs = [round(x[0], 3) for x in runs]
        finally:
            del keep[:]
            for c in ctxs:
                c.close()
        secs = res["seconds"]
        from disq_amd import parallel as P
        dg = [0] * len(res["digests"])
        for p0, d in exported["digests"]:  # the partition digests of the exported host batches
            for i, x in enumerate(d):
                dg[p0 + i] = int(x)
        exported_digest = P.fold_digest(dg)
        out = {"seconds": round(secs, 3),
               "seconds_of_timed_reads": all_secs,
               "decompressed_gbs": round(res["owned_bytes"] / secs / 1e9, 3),
               "reads_per_s": round(exported["records"] / secs, 1),
               "windows": res["windows"], "depth": args.e2e_depth,
               "window_gb": args.e2e_window_gb,
               "stage_seconds_summed_over_windows": {
                   "open_h2d": round(res["open_s"], 3), "pipeline": round(res["run_s"], 3),
                   "d2h_soa_raw": round(res["on_window_s"], 3)},
               "overlap": round((res["open_s"] + res["run_s"] + res["on_window_s"]) / secs, 2),
               "records": exported["records"], "raw_gb": round(exported["raw"] / 1e9, 3),
               "soa_gb": round(exported["soa"] / 1e9, 3),
               "export_mode": args.e2e_export,
               "digest": f"{res['digest']:016x}",
               "digest_match": None if resident_digest is None else res["digest"] == resident_digest,
               "exported_digest_match": exported_digest == res["digest"],
               "setup_s_untimed": round(setup_s, 2),
               "warmup_pass_s_untimed": round(warm_s, 3),
               "arena_gb_per_context": round(arena / 1e9, 2),
               "path": "page cache (/dev/shm) -> pinned staging (16 pread threads per piece, "
                       "double-buffered with the H2D copies) -> HBM -> pipeline -> host SoA + raw "
                       "bytes (lean: + voffsets only) by DMA into a pinned arena, windows of "
                       "whole partitions on "
                       "overlapping contexts (disq_amd.stream + dq_open_shard_path + dq_read)"}
        try:  # the link's ceiling and how close the read comes to it
            pc = pcie_ceiling()
            h2d_b, d2h_b = len(data), exported["raw"] + exported["soa"]
            bound = max(h2d_b / (pc["h2d_gbs"] * 1e9), d2h_b / (pc["d2h_gbs"] * 1e9),
                        (h2d_b + d2h_b) / (pc["bidirectional_gbs"] * 1e9))
            pc.update({"h2d_bytes": h2d_b, "d2h_bytes": d2h_b,
                       "link_bound_s": round(bound, 3),
                       "frac_of_link_bound": round(bound / secs, 3)})
            out["pcie_ceiling"] = pc
        except Exception as e:  # noqa: BLE001
            out["pcie_ceiling"] = {"error": f"{type(e).__name__}: {e}"}
        return out
    except Exception as e:  # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass


if __name__ == "__main__":
    main()
