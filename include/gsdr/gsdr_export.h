/*
 * gsdr-mi355x: symbol visibility. The reference generates this header with CMake's
 * GenerateExportHeader (reference CMakeLists.txt:52-65); here it is written by hand.
 * libgsdr.so is built with -fvisibility=hidden, so only GSDR_PUBLIC entry points are exported.
 */
#ifndef GSDR_EXPORT_H_
#define GSDR_EXPORT_H_

#if defined(GSDR_STATIC_DEFINE)
#define GSDR_PUBLIC
#else
#define GSDR_PUBLIC __attribute__((visibility("default")))
#endif

#endif /* GSDR_EXPORT_H_ */
