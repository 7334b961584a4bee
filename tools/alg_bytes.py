#!/usr/bin/env python3
"""Algorithmic bytes per launch of a bench.py config:
payload bytes + output CRCs (+ the offsets table)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from tools_shapes import SHAPES  # noqa: E402
from mercury_amd.workload import varlen_offsets  # noqa: E402

method, count, length, seed = SHAPES[sys.argv[1]]
w = 4 if method == "crc32c" else 8
if sys.argv[1] == "msgs":  # messages read (headers included), 1 status byte each, the offsets table
    print(int(varlen_offsets(seed, count)[-1]) + count + 8 * (count + 1))
elif sys.argv[1] == "xdr":  # XDR messages read, output CRCs, the offsets table
    import bench
    print(int(bench.xdr_offsets(seed, count)[-1]) + w * count + 8 * (count + 1))
elif sys.argv[1] == "seg":  # bulk-segment layout: + segment table (addr, len) and object index
    print(count * length + w * count + 16 * 4 * count + 8 * (count + 1))
elif length is None:
    print(int(varlen_offsets(seed, count)[-1]) + w * count + 8 * (count + 1))
else:
    print(count * length + w * count)
