#!/usr/bin/env python3
"""A/B build: rv_depth3.py plus kRvWaves = N.  usage: rv_waves_depth3.py KERNELS_HIP N"""
import subprocess,sys
p=sys.argv[1]; n=sys.argv[2]
subprocess.check_call([sys.executable,__import__('os').path.join(__import__('os').path.dirname(__file__), 'rv_depth3.py'),p])
s=open(p).read(); old="constexpr int kRvWaves = 8;"; assert s.count(old)==1
open(p,'w').write(s.replace(old,"constexpr int kRvWaves = %s;"%n))
