/*
 * libds2hip test hooks — NOT part of the product ABI (include/ds2hip.h).
 *
 * Entry points the GPU tests and profiling scripts use to observe the kernels from the
 * outside: holding CUs the way a collective's CTAs would, stamping the device clock, and
 * per-phase clock stamps of the beam search.  Nothing on the training or decoding path
 * calls them; they are exported from the same libds2hip.so so the tests exercise the
 * shipped binary.
 */
#ifndef DS2HIP_TEST_H
#define DS2HIP_TEST_H

#include "ds2hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Residency test hooks (csrc/residency.hip; not on the training path).  ds2_test_occupy:
 * `ctas` one-wave workgroups with lds_kb KB of dynamic LDS each (> 80: alone on their CU,
 * no recurrence workgroup fits beside), each spinning for max_us microseconds on the
 * device clock, recording rec[4*i..4*i+3] = {start, end (s_memrealtime, 100 MHz),
 * XCC id, HW_ID}.  ds2_test_rnn_launch_lds: the same with 94 KB of static LDS launched
 * through the recurrences' launcher and its 80 KB pad (the pad must be clamped to fit).
 * ds2_test_timestamp: *out = s_memrealtime when the stream reaches it.         */
ds2_status_t ds2_test_occupy(int ctas, int lds_kb, int max_us, unsigned long long* rec,
                             ds2_stream_t stream);
ds2_status_t ds2_test_rnn_launch_lds(int ctas, int max_us, unsigned long long* rec,
                                     ds2_stream_t stream);
ds2_status_t ds2_test_timestamp(unsigned long long* out, ds2_stream_t stream);

/* ds2_test_ring_traffic: the local HBM traffic of a ring all-reduce of `count` fp32 values
 * over `world` ranks, on ONE GPU (DESIGN.md §6 interference measurement): 2 (world - 1)
 * phases, each reading a count / world chunk of `bucket` (never written) and of `scratch`
 * (>= count / world floats) and writing the scratch chunk, phase p starting p * (chunk bytes
 * / busbw) after the start (busbw_gbps = 0: unpaced), on `ctas` workgroups of 256 threads.
 * bucket and scratch 16-B aligned.                                                      */
ds2_status_t ds2_test_ring_traffic(const float* bucket, int64_t count, int world, float* scratch,
                                   int ctas, double busbw_gbps, ds2_stream_t stream);

/* ds2_test_beam_stamps: test hook; every later beam decode writes per-phase clock stamps of
 * utterance 0's first 256 frames into buf ([256][9] uint64: s_memtime at the 8 phase
 * boundaries of a frame, then s_memrealtime at its start); buf = NULL turns it off.       */
ds2_status_t ds2_test_beam_stamps(unsigned long long* buf);

#ifdef __cplusplus
}
#endif

#endif /* DS2HIP_TEST_H */
