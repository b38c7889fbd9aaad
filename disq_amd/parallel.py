"""Multi-GPU BAM read: one file, byte-range shards, one process per GPU.

Disq's unit of parallelism is the byte split (one Spark partition per split,
D/impl/formats/sam/AbstractBinarySamSource.java:61-73).  Here the splits of ONE file are dealt in
contiguous groups to the ranks of a torch.distributed process group (RCCL on MI355X, gloo in the
CPU tests).  Rank r holds a resident byte range [O_r, O_{r+1}) of the file (an even share of the
file by default, or the range a rank generated or was placed with) and owns the partitions whose
split starts there (shard_plan).  It decodes [lo_r, hi_r + halo) -- its splits plus a halo that
holds the last partition's straddling record -- with dq_open_shard / dq_open_shard_device.

Exchanges between ranks:
  * the decompressed BAM header, read once by rank 0 and broadcast (every partition needs the
    reference dictionary for the record guesser, BamRecordGuesser.java:107-131);
  * the halo: rank r receives exactly the bytes [O_{r+1}, hi_r + halo) from the ranks that hold
    them -- normally its successor's head -- by one batch of point-to-point sends/receives
    (exchange()).  On an nccl group the bytes go HBM -> xGMI -> HBM and land right behind the
    rank's own resident bytes, so the shard is decoded in place; nothing crosses PCIe;
  * a one-int all_reduce(MAX) so that all ranks agree to grow the halo x4 (a straddling record or
    the guesser's 10-record look-ahead runs past it) or to raise the same error;
  * per-partition descriptors (record count, partition digest), all-gathered so every rank can
    fold the whole-file digest in partition order.
`stitch="file"` re-reads the halo from the file instead (single rank, or a shared file system where
re-reading is cheaper than the exchange).
"""
from __future__ import annotations

import bisect
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


def even_offsets(file_len: int, world: int) -> List[int]:
    """Resident byte ranges [O_r, O_{r+1}) of equal size (O_0 = 0, O_world = file_len)."""
    return [-(-r * file_len // world) for r in range(world)] + [file_len]


def shard_plan(file_len: int, world: int, offsets: Optional[Sequence[int]] = None,
               **split_opts) -> List[Shard]:
    """Contiguous groups of partitions, one per rank: partition p goes to the rank whose resident
    byte range [O_r, O_{r+1}) holds the split's first byte (even ranges by default, i.e. balanced
    by compressed bytes; a generated or pre-placed file passes its ranks' actual ranges)."""
    if offsets is None:
        offsets = even_offsets(file_len, world)
    if len(offsets) != world + 1 or offsets[0] != 0 or offsets[-1] != file_len or \
            any(offsets[i] > offsets[i + 1] for i in range(world)):
        raise ValueError("offsets must be world + 1 non-decreasing values from 0 to file_len")
    sp = path_splits(file_len, **split_opts)
    owner = [min(world - 1, max(0, bisect.bisect_right(offsets, s) - 1)) for s, _ in sp]
    out = []
    for r in range(world):
        ps = [i for i, o in enumerate(owner) if o == r]
        if ps:
            out.append(Shard(r, ps[0], ps[-1] + 1, sp[ps[0]][0], sp[ps[-1]][1]))
        else:
            out.append(Shard(r, 0, 0, 0, 0))
    return out


def halo_transfers(shards: Sequence[Shard], offsets: Sequence[int], file_len: int,
                   halo: int) -> List[Tuple[int, int, int, int]]:
    """(src, dst, a, b): the file bytes [a, b) rank src sends to rank dst.  Rank r decodes
    [lo_r, hi_r + halo) and holds [O_r, O_{r+1}) itself (lo_r >= O_r), so it needs
    [O_{r+1}, hi_r + halo) from the ranks after it: its successor's head, unless that rank's
    range is shorter.  Ordered by destination, then source (file order)."""
    out = []
    for r, s in enumerate(shards):
        if s.empty:
            continue
        a, b = offsets[r + 1], min(file_len, s.hi + halo)
        for q in range(r + 1, len(shards)):
            x, y = max(a, offsets[q]), min(b, offsets[q + 1])
            if x < y:
                out.append((q, r, x, y))
    return out


def exchange(own, offsets: Sequence[int], shards: Sequence[Shard], rank: int, halo: int,
             file_len: int, group=None, out=None):
    """Point-to-point halo exchange (one batch of isend/irecv, no gather): rank r receives the
    file bytes [O_{r+1}, hi_r + halo) from the ranks holding them and sends its own bytes to the
    ranks that need them.  `own` is a uint8 tensor holding [O_r, O_{r+1}); on an nccl group it
    lives in HBM and the bytes cross xGMI device to device (RCCL), never the host.  The received
    bytes, in file order, go to `out` (a uint8 tensor of the right length, e.g. the space right
    behind the own bytes in a resident buffer) or to a new tensor, which is returned."""
    import torch
    import torch.distributed as dist
    tr = halo_transfers(shards, offsets, file_len, halo)
    n = sum(b - a for _, r, a, b in tr if r == rank)
    if out is None:
        out = torch.empty(n, dtype=torch.uint8, device=own.device)
    elif out.numel() != n:
        raise ValueError(f"receive buffer holds {out.numel()} bytes, the halo needs {n}")

    def peer(q):
        return q if group is None else dist.get_global_rank(group, q)
    ops, pos = [], 0
    for q, r, a, b in tr:
        if r == rank:
            ops.append(dist.P2POp(dist.irecv, out[pos:pos + b - a], peer(q), group))
            pos += b - a
        if q == rank:
            ops.append(dist.P2POp(dist.isend, own[a - offsets[q]:b - offsets[q]], peer(r), group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
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
    """Decode one shard on a GPU through dq_open_shard / dq_plan / dq_read.  `data` is host bytes
    or a (device pointer, length) pair of bytes already in this device's memory, followed by 4096
    zero bytes (dq_open_shard_device)."""
    from . import _lib

    def decode(data, base: int, file_len: int, shard: Shard, header: bytes, with_raw: bool):
        with _lib.Context(split_size=split_opts.get("split_size", 0),
                          use_nio=split_opts.get("use_nio", False),
                          hadoop_block_size=split_opts.get("hadoop_block_size", 0),
                          verify_crc=verify_crc, device=device) as c:
            if isinstance(data, tuple):
                c.open_shard_device(data[0], data[1], base, file_len, shard.p0, shard.p1, header)
            else:
                c.open_shard(data, base, file_len, shard.p0, shard.p1, header)
            plan = c.plan()
            b = c.read(with_raw=with_raw)
        nonempty = [shard.p0 + i for i, (_, _, ch) in enumerate(plan) if ch is not None]
        return b, nonempty

    decode.accepts_device = True
    return decode


def _result(shard: Shard, batch: dict, idx: List[int], halo: int) -> ShardResult:
    n = shard.p1 - shard.p0
    counts, digests = [0] * n, [0] * n
    po, pd = batch["part_offset"], batch["part_digest"]
    for k, p in enumerate(idx):
        counts[p - shard.p0] = int(po[k + 1] - po[k])
        digests[p - shard.p0] = int(pd[k])
    return ShardResult(shard, batch, idx, counts, digests, halo)


def read_shard(read_bytes: Callable[[int, int], bytes], file_len: int, shard: Shard,
               header: bytes, decoder, halo: int = 4 << 20, with_raw: bool = False) -> ShardResult:
    """Decode one shard from the file alone (its halo re-read from the file), growing the halo
    when the last partition's record runs past it."""
    from ._lib import DqError
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
    return _result(shard, batch, idx, halo)


class ResidentShard:
    """A rank's resident byte range [O_r, O_{r+1}) in one device buffer with room behind it for
    the halo, so received bytes land right after the own bytes and the library decodes the shard
    in place (dq_open_shard_device).  4096 zero bytes always follow the received ones."""

    def __init__(self, own, device):
        import torch
        self.n_own = int(own.numel()) if hasattr(own, "numel") else len(own)
        self.dev = device
        self.cap = -1
        self._own = own
        self.buf = None
        self.nrecv = 0

    def reserve(self, nrecv: int):
        import torch
        if nrecv > self.cap:
            buf = torch.zeros(self.n_own + nrecv + 4096, dtype=torch.uint8, device=self.dev)
            if self.buf is not None:
                buf[:self.n_own].copy_(self.buf[:self.n_own])
            elif hasattr(self._own, "numel"):
                buf[:self.n_own].copy_(self._own)
            elif self.n_own:
                buf[:self.n_own].copy_(torch.frombuffer(bytearray(self._own), dtype=torch.uint8))
            self._own = None
            self.buf, self.cap = buf, nrecv
        self.nrecv = nrecv
        self.buf[self.n_own + nrecv:self.n_own + nrecv + 4096].zero_()

    @property
    def own(self):
        return self.buf[:self.n_own]

    @property
    def recv(self):
        return self.buf[self.n_own:self.n_own + self.nrecv]

    def span(self, skip: int):
        """(device pointer, length) of the shard data: own bytes from `skip` + the halo."""
        return self.buf.data_ptr() + skip, self.n_own - skip + self.nrecv


def read_shard_exchange(own: bytes, offsets: Sequence[int], file_len: int,
                        shards: Sequence[Shard], rank: int, header: bytes, decoder,
                        halo: int = 4 << 20, with_raw: bool = False, group=None,
                        device: Optional[int] = None) -> ShardResult:
    """Collective form of read_shard: this rank holds the file bytes [O_r, O_{r+1}) (`own`) and
    the halo comes from the next ranks by exchange().  On an nccl group with a decoder that
    accepts device memory the own bytes are placed in HBM once and the halo lands right behind
    them (ResidentShard).  Every rank of `group` must call it; the halo grows x4 on all ranks
    until every shard decodes."""
    import torch
    import torch.distributed as dist
    from ._lib import DqError
    shard = shards[rank]
    o0, o1 = offsets[rank], offsets[rank + 1]
    if len(own) != o1 - o0:
        raise ValueError("own bytes do not match the rank's resident range")
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", device if device is not None else torch.cuda.current_device()) \
        if on_gpu else torch.device("cpu")
    in_place = on_gpu and getattr(decoder, "accepts_device", False)
    res = ResidentShard(own, dev) if in_place else None
    mine = None if in_place else (
        torch.frombuffer(bytearray(own), dtype=torch.uint8) if own else
        torch.zeros(0, dtype=torch.uint8)).to(dev)
    done, err, result = shard.empty, None, None
    while True:
        nrecv = sum(b - a for _, r, a, b in halo_transfers(shards, offsets, file_len, halo)
                    if r == rank)
        if in_place:
            res.reserve(nrecv)
            exchange(res.own, offsets, shards, rank, halo, file_len, group, out=res.recv)
        else:
            got = exchange(mine, offsets, shards, rank, halo, file_len, group)
        status = 0
        if not done:
            try:
                if in_place:
                    torch.cuda.synchronize(dev)
                    data = res.span(shard.lo - o0)
                else:
                    data = own[shard.lo - o0:] + got.cpu().numpy().tobytes()
                result = decoder(data, shard.lo, file_len, shard, header, with_raw)
                done = True
            except DqError as e:
                if "halo too small" in str(e) and shard.hi + halo < file_len:
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
    return _result(shard, batch, idx, halo)


def fold_digest(digests: Sequence[int], first_index: int = 0) -> int:
    """Whole-file digest from per-split digests in split order (dq_api.hip run_pipeline)."""
    d = 0
    for i, x in enumerate(digests):
        d = (d + mix64(int(x) ^ (((first_index + i + 1) * K_WORD) & M64))) & M64
    return d


def fold_digest_np(digests, first_index: int = 0) -> int:
    """fold_digest over a uint64 array, vectorised (uint64 arithmetic wraps mod 2^64)."""
    import numpy as np
    z = np.asarray(digests, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z ^ (np.arange(first_index + 1, first_index + 1 + len(z), dtype=np.uint64)
                 * np.uint64(K_WORD))
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
        return int(z.sum(dtype=np.uint64))


def broadcast_header(header_reader, read_prefix, file_len: int, rank: int, world: int,
                     group=None) -> bytes:
    """Rank 0 reads the decompressed header from the file's first bytes (growing the prefix) and
    broadcasts it.  (header, error) travel together, so a failure on rank 0 raises on every rank
    instead of leaving the others blocked in the broadcast."""
    import torch.distributed as dist
    hdr = [None]
    err = None
    if rank == 0:
        n = 1 << 20
        while True:
            try:
                hdr[0] = (header_reader(read_prefix(min(file_len, n))), None)
                break
            except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
                if n >= file_len:
                    err = e
                    hdr[0] = (None, f"{type(e).__name__}: {e}")
                    break
                n *= 8
    if world > 1:
        dist.broadcast_object_list(hdr, src=0, group=group)
    header, msg = hdr[0]
    if msg is not None:
        if err is not None:
            raise err
        raise RuntimeError(f"rank 0 could not read the BAM header: {msg}")
    return header


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
    if stitch not in ("exchange", "file"):
        raise ValueError(f"stitch must be 'exchange' or 'file', not {stitch!r}")
    # 1. header: rank 0 reads it from the file's first bytes, everyone receives it
    if header_reader is None:
        from . import _lib

        def header_reader(data):
            with _lib.Context(device=device) as c:
                return c.header_from_prefix(data)
    header = broadcast_header(header_reader, lambda n: read_bytes(0, n), file_len, rank, world,
                              group)
    # 2. this rank's shard: it holds the file bytes [O_r, O_{r+1}) and decodes its partitions
    offsets = even_offsets(file_len, world)
    plan = shard_plan(file_len, world, offsets, **split_opts)
    if world > 1 and stitch == "exchange":
        own = read_bytes(offsets[rank], offsets[rank + 1])
        mine = read_shard_exchange(own, offsets, file_len, plan, rank, header, decoder, halo,
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
