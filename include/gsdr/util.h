/*
 * gsdr-mi355x: linkage helpers shared by every public header.
 *
 * Replaces the reference's include/gsdr/util.h:19-29 (GSDR_C_LINKAGE / GSDR_NO_EXCEPT) with the
 * same meaning: C linkage and noexcept when compiled as C++, nothing when compiled as C.
 */
#ifndef GSDR_UTIL_H_
#define GSDR_UTIL_H_

#ifdef __cplusplus
#define GSDR_C_LINKAGE extern "C"
#define GSDR_NO_EXCEPT noexcept
#else
#define GSDR_C_LINKAGE
#define GSDR_NO_EXCEPT
#endif

#endif /* GSDR_UTIL_H_ */
