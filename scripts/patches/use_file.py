#!/usr/bin/env python3
"""Variant build from a whole kernels.hip kept elsewhere (an A/B candidate or an
older tree's file): copies FILE over the COPY that make_variant.sh passes.
usage: make_variant.sh NAME py scripts/patches/use_file.py FILE"""
import shutil
import sys

shutil.copyfile(sys.argv[2], sys.argv[1])
