"""Multi-GPU path (disq_amd/parallel.py): shard planning, descriptor exchange and shard parity.

CPU tests run the collective orchestration with world_size 2 on gloo, using the oracle as each
rank's decoder (the GPU decoder is exercised by the -m gpu tests below, one shard at a time on a
single device: every shard of a file must reproduce the whole-file decode bit for bit).
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from disq_amd import parallel as P
from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _bam1():
    return open(os.path.join(GOLDEN, "1.bam"), "rb").read()


@pytest.mark.parametrize("n,split,nio", [(597482, 128 * 1024, False), (597482, 40000, False),
                                         (597482, 0, False), (105, 100, False), (111, 100, False),
                                         (597482, 65536, True), (10 * 2 ** 30, 0, False)])
def test_path_splits_match_oracle(n, split, nio):
    assert P.path_splits(n, split, nio) == O.path_splits(n, split, nio)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("n,split", [(597482, 40000), (597482, 14146), (10 * 2 ** 30, 0),
                                     (597482, 0)])
def test_shard_plan_tiles_the_partitions(world, n, split):
    plan = P.shard_plan(n, world, split_size=split)
    splits = P.path_splits(n, split)
    owned = [p for s in plan for p in range(s.p0, s.p1)]
    assert owned == list(range(len(splits)))            # each partition once, in order
    for s in plan:
        if not s.empty:
            assert (s.lo, s.hi) == (splits[s.p0][0], splits[s.p1 - 1][1])
    if len(splits) >= world:
        sizes = [s.hi - s.lo for s in plan]
        assert min(sizes) > 0
        assert max(sizes) - min(sizes) <= 2 * max(e - b for b, e in splits)


def test_fold_digest_definition():
    d = [5, 0, 7]
    want = sum(P.mix64(x ^ ((i + 1) * P.K_WORD) & P.M64) for i, x in enumerate(d)) & P.M64
    assert P.fold_digest(d) == want
    assert P.fold_digest(d[1:], first_index=1) + P.mix64(5 ^ P.K_WORD) & P.M64 == want


def test_fold_digest_np_equals_fold_digest():
    rng = np.random.default_rng(5)
    d = rng.integers(0, 2 ** 63, 373, dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(1)
    assert P.fold_digest_np(d) == P.fold_digest([int(x) for x in d])
    assert P.fold_digest_np(d[7:], first_index=7) == P.fold_digest([int(x) for x in d[7:]], 7)
    assert P.fold_digest_np(np.zeros(0, np.uint64)) == 0


def _oracle_decoder(full: bytes, split: int, need: int = 0):
    """Oracle stand-in for the GPU shard decoder; `need` = halo bytes it demands past the shard
    end (the library's "shard halo too small" error otherwise), to exercise halo growth."""
    ob = O.OracleBam(full)
    plan = ob.plan(split)

    def decode(data, base, file_len, shard, header, with_raw):
        from disq_amd._lib import DqError
        assert data == full[base:base + len(data)] and file_len == len(full)
        if base + len(data) < min(file_len, shard.hi + need):
            raise DqError(-2, "shard halo too small")
        assert header == bytes(_oracle_header(full))
        idx, po, pd = [], [0], []
        for p in range(shard.p0, shard.p1):
            ch = plan[p][2]
            if ch is None:
                continue
            recs = ob.read_chunk(*ch)
            idx.append(p)
            po.append(po[-1] + len(recs))
            pd.append(O.stream_digest(recs["hash"]))
        return {"part_offset": np.array(po, np.int64), "part_digest": np.array(pd, np.uint64)}, idx

    return decode


def _oracle_header(full: bytes) -> bytes:
    u = O.OracleBam(full).inflate_all()
    l_text = int.from_bytes(bytes(u[4:8]), "little")
    p = 8 + l_text
    n_ref = int.from_bytes(bytes(u[p:p + 4]), "little")
    p += 4
    for _ in range(n_ref):
        ln = int.from_bytes(bytes(u[p:p + 4]), "little")
        p += 8 + ln
    return bytes(u[:p])


def _worker(rank, world, port, split, stitch, need, halo, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        full = _bam1()
        mine, summary = P.sharded_read(full, split_size=split,
                                       decoder=_oracle_decoder(full, split, need),
                                       header_reader=lambda prefix: _oracle_header(full),
                                       stitch=stitch, halo=halo)
        q.put((rank, mine.shard.p0, mine.shard.p1, summary, mine.halo))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,split,stitch,need,halo", [
    (2, 40000, "exchange", 0, 4 << 20), (2, 14146, "exchange", 0, 4 << 20),
    (3, 128 * 1024, "exchange", 0, 4 << 20), (2, 40000, "file", 0, 4 << 20),
    # halo growth through repeated exchanges: 1 KiB -> 4 -> 16 -> 64 KiB on every rank
    (3, 40000, "exchange", 50000, 1024),
    # more ranks than the halo window spans: the halo is stitched from several ranks' heads
    (5, 14146, "exchange", 70000, 32768)])
def test_sharded_read_gloo(world, split, stitch, need, halo):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, split, stitch, need, halo, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    full = _bam1()
    parts = O.OracleBam(full).read_partitions(split)
    plan = O.OracleBam(full).plan(split)
    digests, k = [], 0
    for s, e, ch in plan:
        if ch is None:
            digests.append(0)
        else:
            digests.append(O.stream_digest(parts[k]["hash"]))
            k += 1
    want = P.fold_digest(digests)
    summaries = [r[3] for r in sorted(res)]
    for s in summaries:   # identical on every rank
        assert s["digest"] == want
        assert s["n_records"] == sum(len(p) for p in parts)
    owned = sorted((r[1], r[2]) for r in res)
    assert owned[0][0] == 0 and owned[-1][1] == len(plan)
    if need:
        assert max(r[4] for r in res) >= need   # the window grew to what the decoder demanded


def test_even_offsets_plan_matches_first_byte_rule():
    """shard_plan with even resident ranges = partition p to rank floor(start * world / len)."""
    for n, split, world in [(597482, 40000, 3), (10 * 2 ** 30, 0, 8), (597482, 14146, 5)]:
        sp = P.path_splits(n, split)
        plan = P.shard_plan(n, world, split_size=split)
        for s in plan:
            for p in range(s.p0, s.p1):
                assert min(world - 1, sp[p][0] * world // n) == s.rank


def test_halo_transfers_cover_exactly_the_missing_bytes():
    n, split = 10 * 2 ** 20, 1 << 20
    offsets = [0, 3_000_000, 3_100_000, 3_150_000, 9_000_000, n]  # short middle ranges
    plan = P.shard_plan(n, 5, offsets, split_size=split)
    for halo in (4096, 300_000, 8 << 20):
        tr = P.halo_transfers(plan, offsets, n, halo)
        for r, s in enumerate(plan):
            got = sorted((a, b) for q, d, a, b in tr if d == r)
            if s.empty:
                assert not got
                continue
            want_lo, want_hi = offsets[r + 1], min(n, s.hi + halo)
            # contiguous pieces tiling [O_{r+1}, hi + halo), each from the rank that holds it
            pos = want_lo
            for a, b in got:
                assert a == pos
                pos = b
            assert pos == max(want_lo, want_hi) or want_hi <= want_lo
        for q, d, a, b in tr:
            assert offsets[q] <= a < b <= offsets[q + 1] and q > d


def _exchange_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        full = bytes((i * 7 + 3) % 251 for i in range(200_000))
        n = len(full)
        offsets = [0, 50_000, 52_000, 140_000, n]
        plan = P.shard_plan(n, world, offsets, split_size=30_000)
        own = torch.frombuffer(bytearray(full[offsets[rank]:offsets[rank + 1]]), dtype=torch.uint8)
        got = P.exchange(own, offsets, plan, rank, 10_000, n)
        s = plan[rank]
        want = b"" if s.empty else full[offsets[rank + 1]:min(n, s.hi + 10_000)]
        q.put((rank, bytes(got.numpy()) == want, len(want)))
    finally:
        dist.destroy_process_group()


def test_exchange_point_to_point_gloo():
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert sum(n for _, _, n in res) > 0


def _header_fail_worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        def bad(prefix):
            raise ValueError("not a BAM")
        try:
            P.sharded_read(_bam1(), split_size=40000, header_reader=bad,
                           decoder=_oracle_decoder(_bam1(), 40000))
            q.put((rank, "no error"))
        except Exception as e:  # noqa: BLE001
            q.put((rank, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def test_header_failure_raises_on_every_rank():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_header_fail_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res[0][1].startswith("ValueError")
    assert all("not a BAM" in m for _, m in res), res


# ---------------------------------------------------------------------------- GPU
FIELDS = ("voffset", "block_size", "ref_id", "pos", "l_seq", "next_ref_id", "next_pos", "tlen",
          "flag", "bin", "n_cigar", "mapq", "l_read_name", "hash")


def _gpu_whole(data, split):
    from disq_amd import _lib
    with _lib.Context(split_size=split, verify_crc=True) as c:
        c.open_bytes(data)
        b = c.read(with_raw=True)
        st = c.run_resident()
    return b, st


def _check_shards(data, split, world, halo):
    from disq_amd import _lib  # noqa: F401
    whole, st = _gpu_whole(data, split)
    dec = P.gpu_shard_decoder({"split_size": split}, device=0)
    hdr_ctx = _lib.Context()
    header = hdr_ctx.header_from_prefix(data[:1 << 20])
    hdr_ctx.close()
    plan = P.shard_plan(len(data), world, split_size=split)
    got = {f: [] for f in FIELDS}
    raw = []
    digests = []
    for s in plan:
        r = P.read_shard(lambda a, b: data[a:b], len(data), s, header, dec, halo=halo,
                         with_raw=True)
        digests += r.digests
        if s.empty:
            continue
        for f in FIELDS:
            got[f].append(r.batch[f])
        raw.append(r.batch["raw"] if r.batch["raw"] is not None else np.zeros(0, np.uint8))
    for f in FIELDS:
        assert np.array_equal(np.concatenate(got[f]), whole[f]), f
    assert np.array_equal(np.concatenate(raw), whole["raw"])
    assert P.fold_digest(digests) == st.digest
    return plan


@pytest.mark.gpu
@pytest.mark.parametrize("split,world", [(128 * 1024, 2), (40000, 3), (40000, 5), (14146, 4),
                                         (65536, 2)])
def test_1bam_shards_equal_whole_file(split, world):
    _check_shards(_bam1(), split, world, halo=16 * 1024)


@pytest.mark.gpu
def test_synthetic_shards_equal_whole_file():
    from disq_amd import synth
    r = synth.generate(150000, seed=7, nthreads=8)
    _check_shards(r.bam, 1 << 20, 4, halo=8 * 1024)


@pytest.mark.gpu
def test_long_read_shards_grow_the_halo():
    from disq_amd import synth
    r = synth.generate(400, seed=5, shape=synth.LONGREAD, nthreads=8)
    _check_shards(r.bam, 256 * 1024, 3, halo=4 * 1024)


@pytest.mark.gpu
def test_sharded_read_single_rank():
    data = _bam1()
    mine, summary = P.sharded_read(data, split_size=40000)
    _, st = _gpu_whole(data, 40000)
    assert summary["digest"] == st.digest and summary["n_records"] == st.n_records


def _gpu_worker(rank, world, port, path, split, halo, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        mine, summary = P.sharded_read(path, split_size=split, device=0, halo=halo,
                                       stitch="exchange")
        q.put((rank, summary["digest"], summary["n_records"], mine.halo))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,split,halo", [("1bam", 40000, 16 * 1024),
                                             ("longread", 256 * 1024, 4 * 1024)])
def test_sharded_read_exchange_gpu(tmp_path, kind, split, halo):
    """Two ranks on the one GPU of the box (gloo carries the head exchange; the decode is the HIP
    library): the stitched shards reproduce the whole-file digest and count."""
    if kind == "1bam":
        data = _bam1()
    else:
        from disq_amd import synth
        data = synth.generate(400, seed=5, shape=synth.LONGREAD, nthreads=8).bam
    path = tmp_path / "in.bam"
    path.write_bytes(data)
    _, st = _gpu_whole(data, split)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, str(path), split, halo, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, digest, n, _ in res:
        assert digest == st.digest and n == st.n_records
    if kind == "longread":
        assert max(r[3] for r in res) > halo   # the straddling long read forced a larger window


def _check_shards_oracle(data, split, world, halo, device_bytes=False):
    """Every shard decoded alone equals the oracle's partitions (Disq's RDD), field by field."""
    import torch
    from disq_amd import _lib
    ob = O.OracleBam(data)
    oplan = ob.plan(split)
    parts = ob.read_partitions(split)
    pidx = [i for i, (_, _, ch) in enumerate(oplan) if ch is not None]
    want = dict(zip(pidx, parts))
    with _lib.Context() as hc:
        header = hc.header_from_prefix(data[:1 << 20])
    dec = P.gpu_shard_decoder({"split_size": split}, device=0)
    if device_bytes:  # the shard's bytes already in HBM (dq_open_shard_device)
        host_dec = dec

        def dec(d, base, file_len, shard, hdr, with_raw):  # noqa: F811
            t = torch.zeros(len(d) + 4096, dtype=torch.uint8, device="cuda:0")
            t[:len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8).to("cuda:0")
            torch.cuda.synchronize()
            return host_dec((t.data_ptr(), len(d)), base, file_len, shard, hdr, with_raw)
    digests = []
    for s in P.shard_plan(len(data), world, split_size=split):
        r = P.read_shard(lambda a, b: data[a:b], len(data), s, header, dec, halo=halo,
                         with_raw=False)
        digests += r.digests
        for k, p in enumerate(r.part_index):
            lo, hi = int(r.batch["part_offset"][k]), int(r.batch["part_offset"][k + 1])
            assert hi - lo == len(want[p]), (s.rank, p)
            for f in FIELDS:
                assert np.array_equal(r.batch[f][lo:hi], want[p][f]), (s.rank, p, f)
        assert sorted(r.part_index) == [p for p in pidx if s.p0 <= p < s.p1]
    assert P.fold_digest(digests) == P.fold_digest(
        [O.stream_digest(want[p]["hash"]) if p in want else 0 for p in range(len(oplan))])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [4, 8])
def test_wgs_shards_equal_oracle(world):
    """configs[2] shape (30x-WGS-like pairs with an unplaced-unmapped tail), byte-range sharded:
    each shard's records equal the oracle's partitions."""
    from disq_amd import synth
    r = synth.generate(200000, seed=17, nthreads=8, unplaced_fraction=0.005)
    _check_shards_oracle(r.bam, 1 << 20, world, halo=64 * 1024, device_bytes=(world == 8))


def _nccl_worker(path, split, q):
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    try:
        data = open(path, "rb").read()
        n = len(data)
        offsets = [0, n]
        plan = P.shard_plan(n, 1, offsets, split_size=split)
        from disq_amd import _lib
        with _lib.Context() as c:
            header = c.header_from_prefix(data[:1 << 20])
        dec = P.gpu_shard_decoder({"split_size": split}, device=0)
        r = P.read_shard_exchange(data, offsets, n, plan, 0, header, dec, halo=4096,
                                  device=0)
        q.put((P.fold_digest(r.digests), sum(r.counts)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_exchange_path_on_nccl_world1(tmp_path):
    """The RCCL (nccl) branch at world size 1: resident shard in HBM, in-place device decode
    (dq_open_shard_device), status all_reduce over RCCL."""
    data = _bam1()
    path = tmp_path / "in.bam"
    path.write_bytes(data)
    _, st = _gpu_whole(data, 40000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(str(path), 40000, q))
    p.start()
    digest, n = q.get(timeout=100)
    p.join(60)
    assert p.exitcode == 0
    assert digest == st.digest and n == st.n_records


@pytest.mark.gpu
def test_resident_shard_in_place_halo_growth():
    """The in-place RCCL branch of read_shard_exchange without a second GPU: rank 0 of 2 holds
    its bytes in a ResidentShard, the halo lands in `recv` by a device-to-device copy (what the
    nccl irecv does), a halo too small for the straddling record is grown x4 -- reserve()
    reallocates and must keep the own bytes -- and the span decoded in place
    (dq_open_shard_device) equals the oracle's partitions of that shard."""
    import torch
    from disq_amd import _lib, synth
    r = synth.generate(60000, seed=29, nthreads=8, unplaced_fraction=0.005)
    data, split = r.bam, 1 << 20
    n = len(data)
    offsets = [0, n // 2, n]
    plan = P.shard_plan(n, 2, offsets, split_size=split)
    s = plan[0]
    assert not s.empty and s.hi > offsets[1]
    full = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda:0")  # "rank 1's" HBM
    rs = P.ResidentShard(full[:offsets[1]].clone(), torch.device("cuda:0"))
    with _lib.Context(split_size=split) as hc:
        header = hc.header_from_prefix(data[:1 << 20])
    ob = O.OracleBam(data)
    oplan = ob.plan(split)
    parts = iter(ob.read_partitions(split))
    want = {i: next(parts) for i, (_, _, ch) in enumerate(oplan) if ch is not None}
    halo, grown, caps = 256, 0, []
    while True:
        tr = [(a, b) for _, rr, a, b in P.halo_transfers(plan, offsets, n, halo) if rr == 0]
        rs.reserve(sum(b - a for a, b in tr))
        caps.append(rs.cap)
        pos = 0
        for a, b in tr:  # the receive: HBM to HBM
            rs.recv[pos:pos + b - a].copy_(full[a:b])
            pos += b - a
        torch.cuda.synchronize()
        ptr, ln = rs.span(s.lo - offsets[0])
        try:
            with _lib.Context(split_size=split) as c:
                c.open_shard_device(ptr, ln, s.lo, n, s.p0, s.p1, header)
                b = c.read(with_raw=False)
            break
        except _lib.DqError as e:
            assert "halo too small" in str(e)
            halo *= 4
            grown += 1
    assert grown >= 1 and len(set(caps)) >= 2  # the buffer was reallocated at least once
    assert torch.equal(rs.own, full[:offsets[1]])  # the own bytes survived the reallocation
    got = np.concatenate([want[p] for p in range(s.p0, s.p1) if p in want])
    assert len(b["voffset"]) == len(got)
    for f in FIELDS:
        assert np.array_equal(b[f], got[f]), f


@pytest.mark.gpu
def test_unplaced_tail_needs_the_file_end():
    """queryUnmapped reads to the end of the file: a shard that stops earlier refuses
    traverseUnplacedUnmapped instead of returning a cut tail; the last shard runs it, with the
    .bai (AbstractBinarySamSource.java:87 -- no index, no traversal) and equals the oracle."""
    from disq_amd import _lib, synth
    a = synth.generate(20000, seed=5, shape=synth.WGS, bai=True, unplaced_fraction=0.05)
    data, split = a.bam, 200000
    with _lib.Context(split_size=split) as c:
        hdr = c.header_from_prefix(data[:1 << 20])
    plan = [s for s in P.shard_plan(len(data), 2, split_size=split) if not s.empty]
    first, last = plan[0], plan[-1]
    assert first.hi < len(data)
    with _lib.Context(split_size=split) as c:
        c.set_index(a.bai)
        c.open_shard(data[first.lo:min(len(data), first.hi + 65536)], first.lo, len(data),
                     first.p0, first.p1, hdr)
        with pytest.raises(_lib.DqError, match="end of the file"):
            c.read(traversal=(None, True))
    ob = O.OracleBam(data)
    oplan = ob.plan(split)
    parts = ob.read_partitions(split, traversal=(None, True), bai=a.bai)
    pidx = [i for i, (_, _, ch) in enumerate(oplan) if ch is not None]
    want = [p for i, p in zip(pidx, parts) if last.p0 <= i < last.p1]
    want = np.concatenate(want) if want else None
    with _lib.Context(split_size=split) as c:
        c.set_index(a.bai)
        c.open_shard(data[last.lo:], last.lo, len(data), last.p0, last.p1, hdr)
        b = c.read(traversal=(None, True), with_raw=False)
    assert len(want) == 1000 and len(b["voffset"]) == len(want)  # the unplaced tail
    assert np.array_equal(b["voffset"], want["voffset"])


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [1, 3, 8])
def test_decode_file_multi_equals_oracle(tmp_path, ndev):
    """dq_decode_file_multi (whole-node mode in one process): the partitions sharded over
    `ndev` contexts (all on device 0 here; one per GPU on a node) fold to the oracle's digest."""
    from disq_amd import _lib, synth
    r = synth.generate(200000, seed=23, nthreads=8, unplaced_fraction=0.005)
    path = tmp_path / "wgs.bam"
    path.write_bytes(r.bam)
    split = 1 << 20
    ob = O.OracleBam(r.bam)
    oplan = ob.plan(split)
    parts = iter(ob.read_partitions(split))
    dig = [O.stream_digest(next(parts)["hash"]) if ch is not None else 0 for _, _, ch in oplan]
    with _lib.Context(split_size=split) as c:
        m = c.decode_file_multi(str(path), [0] * ndev)
    assert m.n_devices == ndev and m.n_partitions == len(oplan)
    assert m.n_records == sum(len(p) for p in ob.read_partitions(split))
    assert m.digest == P.fold_digest(dig)
    assert m.compressed_bytes == len(r.bam)
    assert m.decompressed_bytes == len(ob.inflate_all())


@pytest.mark.parametrize("world", [2, 3, 5])
def test_oracle_shard_window_equals_whole_file(world):
    """The bench's N > 1 parity oracle (oracle.run_partitions_window): each rank's owned partitions
    read from only its window [lo_r, hi_r + halo) of the file, with the decompressed header handed
    over (the window lacks the file's first blocks), equal the whole-file oracle's; a halo that
    cannot hold a straddling record is an error, not a silent short read."""
    import struct
    import numpy as np
    from oracle import oracle as O
    from disq_amd import synth
    r = synth.generate(120000, seed=17, nthreads=8, unplaced_fraction=0.01)
    bam, L = r.bam, len(r.bam)
    split = 512 * 1024
    splits = O.path_splits(L, split)
    cnt, dig, _ = O.run_partitions(bam, splits, 4)
    u = O.OracleBam(bam).inflate_all().tobytes()
    p = 8 + struct.unpack_from("<i", u, 4)[0]
    nr = struct.unpack_from("<i", u, p)[0]
    p += 4
    for _ in range(nr):
        p += 8 + struct.unpack_from("<i", u, p)[0]
    header = u[:p]
    for s in P.shard_plan(L, world, split_size=split):
        if s.empty:
            continue
        win = bam[s.lo:min(L, s.hi + (4 << 20))]
        c2, d2, _ = O.run_partitions_window(win, s.lo, L, header, splits[s.p0:s.p1], 2)
        assert np.array_equal(c2, cnt[s.p0:s.p1]) and np.array_equal(d2, dig[s.p0:s.p1])
        if s.hi < L - 100:
            with pytest.raises(O.OracleError, match="too short"):
                O.run_partitions_window(bam[s.lo:s.hi + 10], s.lo, L, header, splits[s.p0:s.p1], 2)
