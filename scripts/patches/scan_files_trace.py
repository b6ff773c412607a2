#!/usr/bin/env python3
"""Trace build of cc_scan_files (NOT the shipped library): applies
scan_files_trace_r05.diff to the COPY of engine.hip beside the kernels.hip that
make_variant.sh passes, adding per-batch host timestamps (loop start, drain
done, the drained batch's host function, reads done, enqueued) written to
/tmp/cc_scan_trace.txt.  scripts/trace_files.py drives it.
usage: scripts/make_variant.sh trace py scripts/patches/scan_files_trace.py"""
import os
import subprocess
import sys

d = os.path.dirname(os.path.abspath(sys.argv[1]))
diff = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scan_files_trace_r05.diff")
subprocess.run(["patch", "-s", os.path.join(d, "engine.hip"), diff], check=True)
# make_variant.sh refuses a build whose kernels.hip is unchanged: mark the copy
with open(sys.argv[1], "a") as f:
    f.write("\n// scan_files_trace build\n")
