"""Regenerate the committed golden vectors under tests/golden/ (run from the repo root).

Inputs are the reference's own fixtures, copied verbatim from /root/reference/src/test/resources
(data files, not source):
  1.bam, 1-with-splitting-index.bam.sbi, HiSeq...DIQ.sharded.bam/part-r-00000.bam
    -> hiseq_part-r-00000.bam
Outputs (expected values; every count also appears literally in tests/test_oracle_golden.py):
  golden.json              -- facts asserted by the reference's tests or derived by the oracle
  1.bam.records.npz        -- per-record voffset/block_size/refID/pos/flag/hash of 1.bam
  hiseq.records.npz        -- the same for the HiSeq part

Provenance of each value is recorded in golden.json["provenance"].  Per-record hashes are
oracle-derived ("parity unpinned by reference tests": no reference test compares record bytes);
the oracle itself is pinned by the SBI record starts and block KAT.
"""
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402


def sbi_offsets(path):
    d = open(path, "rb").read()
    assert d[:4] == b"SBI\x01"
    n = struct.unpack_from("<q", d, 60)[0]
    return np.frombuffer(d, "<u8", count=n, offset=68)


def main():
    out = {"provenance": {}}
    b = O.OracleBam.from_path(os.path.join(HERE, "1.bam"))
    blocks = []
    for s, e in O.path_splits(b.len, 128 * 1024):
        blocks += b.split_blocks(s, e)
    out["1.bam"] = {
        "file_len": b.len,
        "n_blocks_128k": len(blocks),
        "block0": list(blocks[0]),
        "n_records": int(len(b.read_all())),
        "partitions_128k": [len(p) for p in b.read_partitions(128 * 1024)],
        "partitions_40000": [len(p) for p in b.read_partitions(40000)],
        "total_split_14146": int(sum(len(p) for p in b.read_partitions(14146))),
        "total_split_19687": int(sum(len(p) for p in b.read_partitions(19687))),
        "decompressed_len": int(len(b.inflate_all())),
    }
    out["provenance"]["1.bam"] = (
        "n_blocks_128k/block0: BgzfBlockSourceTest.java:31-35; n_records: SBI fixture "
        "(totalRecords) and BamRecordGuesserCheckerTest; partitions/totals: oracle-derived")
    recs = b.read_all()
    np.savez_compressed(os.path.join(HERE, "1.bam.records.npz"),
                        voffset=recs["voffset"], block_size=recs["block_size"],
                        ref_id=recs["ref_id"], pos=recs["pos"], flag=recs["flag"],
                        hash=recs["hash"])
    h = O.OracleBam.from_path(os.path.join(HERE, "hiseq_part-r-00000.bam"))
    hr = h.read_all()
    out["hiseq"] = {"n_records": int(len(hr)), "n_unplaced": int((hr["ref_id"] == -1).sum()),
                    "partitions_40000": [len(p) for p in h.read_partitions(40000)]}
    out["provenance"]["hiseq"] = "oracle-derived (no reference test reads this fixture)"
    np.savez_compressed(os.path.join(HERE, "hiseq.records.npz"), voffset=hr["voffset"],
                        hash=hr["hash"])
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
