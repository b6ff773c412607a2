/* include/curve_crc32_compat.h -- drop-in bodies for the reference's two CRC32
 * wrapper headers over libcurvecrc's CPU primitive:
 *   - curve::common::CRC32, src/common/crc32.h:40-55
 *   - nebd::common::CRC32,  nebd/src/common/crc32.h:31-38
 * Same names, overloads and semantics as there (butil::crc32c::Value / Extend):
 *   CRC32(p, n)      == Value(p, n)
 *   CRC32(crc, p, n) == Extend(crc, p, n), so CRC32(CRC32(a), b) == CRC32(a || b).
 * A maintainer replaces the body of either header with an include of this one
 * (INTEGRATION.md section 2).  Define CURVE_CRC32_COMPAT_NO_CURVE or
 * CURVE_CRC32_COMPAT_NO_NEBD to leave a namespace out.  C++ only; the C ABI
 * itself is include/curve_crc.h. */
#ifndef CURVE_CRC32_COMPAT_H_
#define CURVE_CRC32_COMPAT_H_

#ifdef __cplusplus
#include <stddef.h>
#include <stdint.h>

#include "curve_crc.h"

#ifndef CURVE_CRC32_COMPAT_NO_CURVE
namespace curve {
namespace common {
inline uint32_t CRC32(const char* pData, size_t iLen) { return crc32c_value(pData, iLen); }
inline uint32_t CRC32(uint32_t crc, const char* pData, size_t iLen) { return crc32c_extend(crc, pData, iLen); }
}  // namespace common
}  // namespace curve
#endif

#ifndef CURVE_CRC32_COMPAT_NO_NEBD
namespace nebd {
namespace common {
inline uint32_t CRC32(const char* pData, size_t iLen) { return crc32c_value(pData, iLen); }
inline uint32_t CRC32(uint32_t crc, const char* pData, size_t iLen) { return crc32c_extend(crc, pData, iLen); }
}  // namespace common
}  // namespace nebd
#endif

#endif  /* __cplusplus */
#endif  /* CURVE_CRC32_COMPAT_H_ */
