/*
 * gsdr-mi355x umbrella header (reference include/gsdr/gsdr.h:19-30): the hot-path C ABI.
 */
#ifndef GSDR_GSDR_H_
#define GSDR_GSDR_H_

#include <gsdr/am.h>
#include <gsdr/arithmetic.h>
#include <gsdr/conversion.h>
#include <gsdr/cuda_util.h>
#include <gsdr/fir.h>
#include <gsdr/fm.h>
#include <gsdr/gsdr_ext.h>
#include <gsdr/hip_util.h>
#include <gsdr/iir.h>
#include <gsdr/qpsk.h>
#include <gsdr/qpsk256.h>
#include <gsdr/quad_demod.h>
#include <gsdr/stream.h>
#include <gsdr/trig.h>
#include <gsdr/util.h>

#endif /* GSDR_GSDR_H_ */
