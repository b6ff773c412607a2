#!/usr/bin/env python3
"""Round-4 wait_tiles (every waiting wave counts every missing tile itself)
swapped into a COPY of kernels.hip: the A/B baseline of the claim-based
fallback (scripts/concurrent_ranges.py).  usage: wait_tiles_noclaim.py KERNELS_HIP"""
import sys

p = sys.argv[1]
s = open(p).read()
i = s.index("// Every tile count of this call into tb")
j = s.index("// The tile holding unit u of the stream", i)
s = s[:i] + "// Every tile count of this call into tb (lane l: tiles kTpl*l .. kTpl*l + kTpl-1):\n// poll the epoch-tagged words (sc1 loads: a data-tagged granule needs no\n// fence), and count a tile whose word is still missing after kTileWaitTicks\n// with count(t) -- its workgroup is not running, and no wave waits on another\n// without a bound.\ntemplate <int kTpl, typename Count>\n__device__ __forceinline__ void wait_tiles(uint64_t (&tb)[kTpl], uint64_t* tiles, uint64_t tag, uint32_t lane,\n                                           Count count) {\n    constexpr uint64_t kCountMask = (1ull << kEpochShift) - 1;\n    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();\n    uint32_t have = 0;  // bit j: tb[j] holds this call's count\n    for (;;) {\n#pragma unroll\n        for (int j = 0; j < kTpl; j++) {\n            const uint64_t v = __hip_atomic_load(tiles + kTpl * lane + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n            const bool ok = (v & ~kCountMask) == tag;\n            tb[j] = ok ? v & kCountMask : tb[j];\n            have |= ok ? 1u << j : 0u;\n        }\n        if (!__ballot(have != (1u << kTpl) - 1u)) return;\n        if (__builtin_amdgcn_s_memrealtime() - t0 > kTileWaitTicks) break;\n        __builtin_amdgcn_s_sleep(2);\n    }\n#pragma unroll\n    for (int j = 0; j < kTpl; j++) {\n        for (uint64_t m = __ballot(!((have >> j) & 1u)); m; m &= m - 1) {\n            const uint32_t l = (uint32_t)__builtin_ctzll(m);\n            const uint64_t cnt = count(kTpl * l + j);\n            tb[j] = lane == l ? cnt : tb[j];\n        }\n    }\n}\n\n" + s[j:]
open(p, "w").write(s)
