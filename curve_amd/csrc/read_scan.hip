// curve_amd/csrc/read_scan.hip -- the one library primitive of the batched
// paths, called on rocPRIM directly: the exclusive scan that lays out the page
// slots of a batch of reads (cc_verify_reads_dev).  Kept in its own
// translation unit: the template instantiations are heavy and nothing else
// here needs them.  (The write log groups its pieces with a device hash table,
// log_insert_kernel, and needs no sort.)
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>

#include "kernels.h"

namespace cc {

size_t scan_temp_bytes(uint64_t n) {
    size_t bytes = 0;
    // sizing query only (no launch)
    if (rocprim::exclusive_scan(nullptr, bytes, static_cast<const uint64_t*>(nullptr), static_cast<uint64_t*>(nullptr),
                                uint64_t(0), (size_t)n, rocprim::plus<uint64_t>()) != hipSuccess)
        return 0;
    return bytes;
}

hipError_t exclusive_scan_u64(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out, uint64_t n,
                              hipStream_t s) {
    size_t bytes = temp_bytes;
    return rocprim::exclusive_scan(temp, bytes, in, out, uint64_t(0), (size_t)n, rocprim::plus<uint64_t>(), s);
}

}  // namespace cc
