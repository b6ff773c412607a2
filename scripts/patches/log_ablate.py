#!/usr/bin/env python3
"""Timing-ablation build of the write-log page kernel (NOT the shipped kernel;
wrong results by design): patches a COPY of kernels.hip so that chosen memory
streams of the page step pass out-of-range buffer offsets (every instruction
still issues; the buffer unit returns 0 / drops the store without touching
memory).  Metadata loads (head records, table entries, descriptors, links) and
the CRC stores stay.
usage: log_ablate.py KERNELS_HIP MODE   MODE: nodata | nostores | nopage | nosrc"""
import sys

p, mode = sys.argv[1], sys.argv[2]
s = open(p).read()


def in_func(name, old, new):
    """replace every `old` inside the body of the function that starts at `name`"""
    global s
    a = s.index(name)
    b = s.index("\n}\n", a)
    body = s[a:b]
    assert old in body, (name, old)
    s = s[:a] + body.replace(old, new) + s[b:]


if mode in ("nodata", "nopage"):
    # nopage: the rows read from the page go out of range (covered rows still come from the source)
    in_func("__device__ __forceinline__ void load_rows_sel(", "row_sel(4u * lane)",
            "row_sel(kBufOOB)" if mode == "nodata" else "row_sel(((cov >> j) & 1u) ? 4u * lane : kBufOOB)")
    in_func("__device__ __forceinline__ void load_rows(", "row_sel(((rows >> j) & 1u) ? 4u * lane : kBufOOB)",
            "row_sel(kBufOOB)")
if mode in ("nodata", "nosrc"):
    for f in ("__device__ __forceinline__ void fetch_edges(", "__device__ __forceinline__ void fetch_piece("):
        in_func(f, "(mine && k0 < 4u - sh) ? b : kBufOOB", "kBufOOB")
        in_func(f, "(mine && sh && k1 > 4u - sh) ? b + 4 : kBufOOB", "kBufOOB")
    in_func("__device__ __forceinline__ void fetch_edges(", "in ? 4u * lane + 256u * r.r[q] : kBufOOB", "kBufOOB")
    in_func("__device__ __forceinline__ void fetch_piece(", "row_sel(full ? l4 : kBufOOB)", "row_sel(kBufOOB)")
    if mode == "nosrc":  # covered rows read from the page instead of the source
        in_func("__device__ __forceinline__ void load_rows_sel(", "((cov >> j) & 1u) ? rs : rp", "rp")
if mode in ("nodata", "nostores"):
    in_func("__device__ __forceinline__ void log_pages_body(", "row_sel(((dirty >> j) & 1u) ? 4u * lane : kBufOOB)",
            "row_sel(kBufOOB)")
open(p, "w").write(s)
