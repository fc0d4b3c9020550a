// HIP streams with a chosen hardware-queue placement.
//
// A process gets GPU_MAX_HW_QUEUES hardware queues per device (4 on the MI355X boxes; HIP's
// default) and HIP multiplexes every ordinary stream onto them: two streams that land on the same
// queue execute one after the other, whatever their events say.  Measured in the device-resident
// pipeline (tools/gpu_r3_streams_trace.sh, rocprofv3 Queue_Id): the consumer's two peak-finder
// streams shared one queue, and with two producer streams the peak finder shared the producers'
// queues -- launches meant to overlap were serialised.  A stream created with a CU mask owns its
// hardware queue (the mask is a queue property); an all-CUs mask restricts nothing.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pr {

enum StreamKind { kStreamShared = 0, kStreamDedicated = 1, kStreamHighPriority = 2 };
hipStream_t make_stream(int device, int kind);
// Streams with a placement (dedicated / high priority) come from a process-wide pool per (device,
// kind) and go back to it: a hardware queue of its own is a scarce per-process resource, and such
// streams are never destroyed while the process runs.  Ordinary streams are created and destroyed.
hipStream_t acquire_stream(int device, int kind);
void release_stream(int device, int kind, hipStream_t s);   // synchronises s first
// Process exit (after the native threads halted): destroy the pooled streams; streams released
// afterwards are destroyed at once.  Leaves no queue of ours to the runtime's static teardown, which
// a profiler's own teardown (rocprofv3) does not survive.
void close_stream_pool();

}  // namespace pr
