"""Multi-GPU BAM read: one file, byte-range shards, one process per GPU.

Disq's unit of parallelism is the byte split (one Spark partition per split,
D/impl/formats/sam/AbstractBinarySamSource.java:61-73).  Here the splits of ONE file are dealt in
contiguous groups to the ranks of a torch.distributed process group (RCCL on MI355X, gloo in the
CPU tests), balanced by compressed bytes.  Each rank reads its group's bytes plus a halo that
holds the last partition's straddling record, decodes them with dq_open_shard, and the ranks
exchange two small messages:
  * the decompressed BAM header, read once by rank 0 and broadcast (every partition needs the
    reference dictionary for the record guesser, BamRecordGuesser.java:107-131);
  * per-partition descriptors (record count, partition digest, first record pointer), all-gathered
    so every rank can fold the whole-file digest in partition order and check that the shards
    tile the file exactly as the single-GPU stream does.
Shard boundary stitching (north star): a record that starts in a rank's last
partition may run into the next rank's bytes.  With `stitch="exchange"` (the default for world > 1)
every rank reads only its own byte range from the file and the halo is assembled from an
all_gather of every shard's first `halo` compressed bytes (RCCL over xGMI when the group's backend
is nccl, gloo on CPU); rank r appends the heads of ranks r+1, r+2, ... until it holds `halo` bytes
past its end.  When a rank's straddling record (or the guesser's 10-record look-ahead) needs more,
all ranks agree through a one-int all_reduce and repeat the exchange with a 4x larger window.
`stitch="file"` reads the halo from the file instead (single rank, or a shared file system where
re-reading is cheaper than the exchange).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

M64 = (1 << 64) - 1
K_LEN = 0x9E3779B97F4A7C15
K_WORD = 0xD6E8FEB86659FD93


def mix64(z: int) -> int:
    """splitmix64 finaliser (dq_internal.h dq_mix64)."""
    z &= M64
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return z


def path_splits(file_len: int, split_size: int = 0, use_nio: bool = False,
                hadoop_block_size: int = 0) -> List[Tuple[int, int]]:
    """PathSplitSource.getPathSplits (D/impl/file/PathSplitSource.java:26-64) for one file: NIO
    ceil(len/splitSize) splits (:32-42) or Hadoop 2.7 FileInputFormat.getSplits (:44-62,
    SPLIT_SLOP 1.1, split size = min(splitSize, block size), 32 MiB local blocks)."""
    if use_nio:
        if split_size <= 0:
            raise ValueError("splitSize must be > 0 with useNio")
        n = (file_len + split_size - 1) // split_size
        return [(i * split_size, min(file_len, (i + 1) * split_size)) for i in range(n)]
    block = hadoop_block_size if hadoop_block_size > 0 else 32 * 1024 * 1024
    ss = max(1, min(split_size if split_size > 0 else (1 << 62), block))
    if file_len == 0:
        return [(0, 0)]
    out, rem = [], file_len
    while rem / ss > 1.1:
        out.append((file_len - rem, file_len - rem + ss))
        rem -= ss
    if rem:
        out.append((file_len - rem, file_len))
    return out


@dataclass(frozen=True)
class Shard:
    rank: int
    p0: int          # first partition (split index) owned
    p1: int          # one past the last
    lo: int          # first byte of split p0
    hi: int          # end of split p1 - 1

    @property
    def empty(self):
        return self.p1 <= self.p0


def shard_plan(file_len: int, world: int, **split_opts) -> List[Shard]:
    """Contiguous groups of partitions, one per rank, balanced by compressed bytes: partition p
    goes to the rank whose 1/world slice of the file holds the split's first byte."""
    sp = path_splits(file_len, **split_opts)
    owner = [min(world - 1, (s * world) // max(1, file_len)) for s, _ in sp]
    out = []
    for r in range(world):
        ps = [i for i, o in enumerate(owner) if o == r]
        if ps:
            out.append(Shard(r, ps[0], ps[-1] + 1, sp[ps[0]][0], sp[ps[-1]][1]))
        else:
            out.append(Shard(r, 0, 0, 0, 0))
    return out


@dataclass
class ShardResult:
    shard: Shard
    batch: dict                 # dq_read batch (SoA fields, raw bytes, part_offset, part_digest)
    part_index: List[int]       # global split index of each non-empty partition in `batch`
    counts: List[int]           # records per owned split (p0..p1-1), empty ones included
    digests: List[int]          # digest per owned split (0 when empty)
    halo: int


def gpu_shard_decoder(split_opts: dict, device: int, verify_crc: bool = True):
    """Decode one shard on a GPU through dq_open_shard / dq_plan / dq_read."""
    from . import _lib

    def decode(data: bytes, base: int, file_len: int, shard: Shard, header: bytes, with_raw: bool):
        with _lib.Context(split_size=split_opts.get("split_size", 0),
                          use_nio=split_opts.get("use_nio", False),
                          hadoop_block_size=split_opts.get("hadoop_block_size", 0),
                          verify_crc=verify_crc, device=device) as c:
            c.open_shard(data, base, file_len, shard.p0, shard.p1, header)
            plan = c.plan()
            b = c.read(with_raw=with_raw)
        nonempty = [shard.p0 + i for i, (_, _, ch) in enumerate(plan) if ch is not None]
        return b, nonempty

    return decode


def read_shard(read_bytes: Callable[[int, int], bytes], file_len: int, shard: Shard,
               header: bytes, decoder, halo: int = 4 << 20, with_raw: bool = False) -> ShardResult:
    """Decode one shard, growing the halo when the last partition's record runs past it."""
    from ._lib import DqError
    n = shard.p1 - shard.p0
    if shard.empty:
        return ShardResult(shard, {}, [], [], [], 0)
    while True:
        end = min(file_len, shard.hi + halo)
        data = read_bytes(shard.lo, end)
        try:
            batch, idx = decoder(data, shard.lo, file_len, shard, header, with_raw)
            break
        except DqError as e:
            if "halo too small" in str(e) and end < file_len:
                halo *= 4
                continue
            raise
    counts, digests = [0] * n, [0] * n
    po, pd = batch["part_offset"], batch["part_digest"]
    for k, p in enumerate(idx):
        counts[p - shard.p0] = int(po[k + 1] - po[k])
        digests[p - shard.p0] = int(pd[k])
    return ShardResult(shard, batch, idx, counts, digests, halo)


def _halo_from_heads(heads: Sequence[bytes], shards: Sequence[Shard], rank: int, halo: int) -> bytes:
    """File bytes [hi_rank, hi_rank + halo) from the gathered shard heads: head k holds
    min(halo, hi_k - lo_k) bytes starting at lo_k, and shards tile the file in rank order."""
    out, need = [], halo
    for k in range(rank + 1, len(shards)):
        if shards[k].empty:
            continue
        h = heads[k]
        out.append(h[:need])
        need -= min(need, len(h))
        if need == 0 or len(h) < shards[k].hi - shards[k].lo:
            break
    return b"".join(out)


def exchange_heads(own: bytes, shards: Sequence[Shard], rank: int, halo: int, group=None,
                   device: Optional[int] = None) -> bytes:
    """all_gather of every shard's first `halo` bytes (fixed-size window, one collective); returns
    this rank's halo.  On an nccl (RCCL) group the window lives in HBM and crosses xGMI."""
    import torch
    import torch.distributed as dist
    world = len(shards)
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", device if device is not None else torch.cuda.current_device()) \
        if on_gpu else torch.device("cpu")
    mine = torch.zeros(halo, dtype=torch.uint8)
    head = own[:halo]
    if head:
        mine[:len(head)] = torch.frombuffer(bytearray(head), dtype=torch.uint8)
    mine = mine.to(dev)
    every = torch.empty(world * halo, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(every, mine, group=group)
    every = every.cpu().numpy()
    heads = [every[k * halo:k * halo + min(halo, max(0, s.hi - s.lo))].tobytes()
             for k, s in enumerate(shards)]
    return _halo_from_heads(heads, shards, rank, halo)


def read_shard_exchange(read_bytes: Callable[[int, int], bytes], file_len: int,
                        shards: Sequence[Shard], rank: int, header: bytes, decoder,
                        halo: int = 4 << 20, with_raw: bool = False, group=None,
                        device: Optional[int] = None) -> ShardResult:
    """Collective form of read_shard: own bytes from the file, halo from exchange_heads.  Every
    rank of `group` must call it; the halo grows x4 on all ranks until every shard decodes."""
    import torch
    import torch.distributed as dist
    from ._lib import DqError
    shard = shards[rank]
    n = shard.p1 - shard.p0
    own = read_bytes(shard.lo, shard.hi) if not shard.empty else b""
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", device if device is not None else torch.cuda.current_device()) \
        if on_gpu else torch.device("cpu")
    done, err, result = shard.empty, None, None
    while True:
        h = exchange_heads(own, shards, rank, halo, group, device)
        status = 0
        if not done:
            try:
                result = decoder(own + h, shard.lo, file_len, shard, header, with_raw)
                done = True
            except DqError as e:
                if "halo too small" in str(e) and shard.hi + len(h) < file_len:
                    status = 1
                else:
                    status, err = 2, e
            except Exception as e:  # noqa: BLE001 -- re-raised below, after the ranks agree
                status, err = 2, e
        flag = torch.tensor([status], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        worst = int(flag.item())
        if worst == 2:
            raise err if err is not None else RuntimeError("sharded read failed on another rank")
        if worst == 0:
            break
        halo *= 4
    if shard.empty:
        return ShardResult(shard, {}, [], [], [], 0)
    batch, idx = result
    counts, digests = [0] * n, [0] * n
    po, pd = batch["part_offset"], batch["part_digest"]
    for k, p in enumerate(idx):
        counts[p - shard.p0] = int(po[k + 1] - po[k])
        digests[p - shard.p0] = int(pd[k])
    return ShardResult(shard, batch, idx, counts, digests, halo)


def fold_digest(digests: Sequence[int], first_index: int = 0) -> int:
    """Whole-file digest from per-split digests in split order (dq_api.hip run_pipeline)."""
    d = 0
    for i, x in enumerate(digests):
        d = (d + mix64(int(x) ^ (((first_index + i + 1) * K_WORD) & M64))) & M64
    return d


def sharded_read(path_or_bytes, split_size: int = 0, use_nio: bool = False,
                 hadoop_block_size: int = 0, device: Optional[int] = None, decoder=None,
                 header_reader=None, with_raw: bool = False, halo: int = 4 << 20, group=None,
                 stitch: str = "exchange"):
    """Collective read of one BAM by all ranks of `group` (torch.distributed).

    Returns (ShardResult of this rank, summary) where summary holds the whole-file record count,
    per-split counts and the whole-file digest (identical on every rank)."""
    import torch.distributed as dist

    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview, np.ndarray)):
        buf = memoryview(path_or_bytes).cast("B")
        file_len = len(buf)

        def read_bytes(a, b):
            return bytes(buf[a:b])
    else:
        path = os.fspath(path_or_bytes)
        file_len = os.path.getsize(path)

        def read_bytes(a, b):
            with open(path, "rb") as f:
                f.seek(a)
                return f.read(b - a)
    split_opts = dict(split_size=split_size, use_nio=use_nio, hadoop_block_size=hadoop_block_size)
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    if decoder is None:
        decoder = gpu_shard_decoder(split_opts, device)
    # 1. header: rank 0 reads it from the file's first bytes, everyone receives it
    hdr = [None]
    if rank == 0:
        if header_reader is None:
            from . import _lib

            def header_reader(data):
                with _lib.Context(device=device) as c:
                    return c.header_from_prefix(data)
        n = 1 << 20
        while True:
            try:
                hdr[0] = header_reader(read_bytes(0, min(file_len, n)))
                break
            except Exception:
                if n >= file_len:
                    raise
                n *= 8
    if world > 1:
        dist.broadcast_object_list(hdr, src=0, group=group)
    header = hdr[0]
    # 2. this rank's shard
    plan = shard_plan(file_len, world, **split_opts)
    if stitch not in ("exchange", "file"):
        raise ValueError(f"stitch must be 'exchange' or 'file', not {stitch!r}")
    if world > 1 and stitch == "exchange":
        mine = read_shard_exchange(read_bytes, file_len, plan, rank, header, decoder, halo,
                                   with_raw, group, device)
    else:
        mine = read_shard(read_bytes, file_len, plan[rank], header, decoder, halo, with_raw)
    # 3. descriptors of every shard
    desc = (mine.shard.p0, mine.counts, mine.digests)
    every = [None] * world
    if world > 1:
        dist.all_gather_object(every, desc, group=group)
    else:
        every = [desc]
    nsplit = len(path_splits(file_len, **split_opts))
    counts, digests = [0] * nsplit, [0] * nsplit
    for p0, cs, ds in every:
        for i, (c, d) in enumerate(zip(cs, ds)):
            counts[p0 + i] = c
            digests[p0 + i] = d
    summary = {"n_records": sum(counts), "counts": counts, "digest": fold_digest(digests),
               "n_partitions": nsplit, "world": world}
    return mine, summary
