// curve_amd/csrc/log_sort.hip -- the library primitives of the batched paths
// (hipCUB over rocPRIM): the stable device radix sort of the write log's
// (page, update index) pieces, and the exclusive scan that lays out the page
// slots of a batch of reads.  Kept in their own translation unit: the template
// instantiations are heavy and nothing else here needs them.
//
// Stability is what carries the raft-log order (op_request.cpp:429-481 applies
// writes in log order): pieces are generated in write order, so after a STABLE
// sort by page the pieces of one page are still in write order and the page
// kernel applies them front to back (later writes win).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <stdint.h>

#include "kernels.h"

namespace cc {

#ifndef CC_SORT_ONESWEEP
#define CC_SORT_ONESWEEP 0  // 1: force rocPRIM's onesweep radix sort (default picks merge sort below 1M keys)
#endif
namespace {
using OnesweepOnly = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;
}

size_t log_sort_temp_bytes(uint64_t n) {
    size_t bytes = 0;
    // sizing query only (no launch); 32 bits is the widest sort ever requested
#if CC_SORT_ONESWEEP
    if (rocprim::radix_sort_pairs<OnesweepOnly>(nullptr, bytes, static_cast<const uint32_t*>(nullptr),
                                                static_cast<uint32_t*>(nullptr), static_cast<const uint32_t*>(nullptr),
                                                static_cast<uint32_t*>(nullptr), (unsigned int)n, 0u, 32u) != hipSuccess)
        return 0;
#else
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, static_cast<const uint32_t*>(nullptr),
                                           static_cast<uint32_t*>(nullptr), static_cast<const uint32_t*>(nullptr),
                                           static_cast<uint32_t*>(nullptr), (int)n, 0, 32) != hipSuccess)
        return 0;
#endif
    return bytes;
}

hipError_t log_sort(void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                    const uint32_t* vals_in, uint32_t* vals_out, uint64_t n, int end_bit, hipStream_t s) {
    size_t bytes = temp_bytes;
#if CC_SORT_ONESWEEP
    return rocprim::radix_sort_pairs<OnesweepOnly>(temp, bytes, keys_in, keys_out, vals_in, vals_out, (unsigned int)n,
                                                   0u, (unsigned int)end_bit, s);
#else
    return hipcub::DeviceRadixSort::SortPairs(temp, bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0, end_bit,
                                              s);
#endif
}

size_t scan_temp_bytes(uint64_t n) {
    size_t bytes = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, static_cast<const uint64_t*>(nullptr),
                                         static_cast<uint64_t*>(nullptr), (int)n) != hipSuccess)
        return 0;
    return bytes;
}

hipError_t exclusive_scan_u64(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out, uint64_t n,
                              hipStream_t s) {
    size_t bytes = temp_bytes;
    return hipcub::DeviceScan::ExclusiveSum(temp, bytes, in, out, (int)n, s);
}

}  // namespace cc
