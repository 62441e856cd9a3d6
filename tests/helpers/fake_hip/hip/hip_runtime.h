/*
 * A CPU stand-in for the part of the HIP runtime that gss_run.hip calls (tools/sanitize.sh
 * builds gss_run.hip against it with -fsanitize=thread and -fsanitize=address,undefined).
 * Test infrastructure only: nothing here runs on a GPU or ships in the library.
 *
 * Streams are in-order queues, each drained by its own host thread, so that the run's host
 * threads and its "device" work interleave as they do on the GPU; events are generation
 * counters; device and pinned memory are host allocations.  Device functions (kernels) are
 * the fakes of tests/helpers/fake_dev.cpp, enqueued on their stream with fake_enqueue.
 */
#ifndef FAKE_HIP_RUNTIME_H
#define FAKE_HIP_RUNTIME_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
#include <functional>
#endif

typedef enum hipError_t {
    hipSuccess = 0,
    hipErrorInvalidValue = 1,
    hipErrorOutOfMemory = 2,
    hipErrorNotReady = 600,
} hipError_t;
typedef enum hipMemcpyKind {
    hipMemcpyHostToHost = 0,
    hipMemcpyHostToDevice = 1,
    hipMemcpyDeviceToHost = 2,
    hipMemcpyDeviceToDevice = 3,
    hipMemcpyDefault = 4,
} hipMemcpyKind;
typedef enum hipDeviceAttribute_t {
    hipDeviceAttributeMultiprocessorCount = 16,
} hipDeviceAttribute_t;
typedef struct fake_stream *hipStream_t;
typedef struct fake_event *hipEvent_t;
#define hipStreamDefault 0u
#define hipStreamNonBlocking 1u
#define hipEventDefault 0u
#define hipEventDisableTiming 2u
#define hipHostMallocDefault 0u

const char *hipGetErrorString(hipError_t e);
hipError_t hipGetLastError(void);
hipError_t hipGetDevice(int *d);
hipError_t hipSetDevice(int d);
hipError_t hipDeviceSynchronize(void);
hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t a, int dev);
hipError_t hipDeviceGetStreamPriorityRange(int *lo, int *hi);
hipError_t hipMalloc(void **p, size_t n);
hipError_t hipFree(void *p);
hipError_t hipHostMalloc(void **p, size_t n, unsigned flags);
hipError_t hipHostFree(void *p);
hipError_t hipMemcpy(void *dst, const void *src, size_t n, hipMemcpyKind k);
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind k, hipStream_t s);
hipError_t hipMemsetAsync(void *dst, int v, size_t n, hipStream_t s);
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned flags);
hipError_t hipStreamCreateWithPriority(hipStream_t *s, unsigned flags, int prio);
hipError_t hipExtStreamCreateWithCUMask(hipStream_t *s, uint32_t n, const uint32_t *mask);
hipError_t hipStreamDestroy(hipStream_t s);
hipError_t hipStreamSynchronize(hipStream_t s);
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned flags);
hipError_t hipEventCreate(hipEvent_t *e);
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned flags);
hipError_t hipEventDestroy(hipEvent_t e);
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s);
hipError_t hipEventSynchronize(hipEvent_t e);
hipError_t hipEventQuery(hipEvent_t e);
hipError_t hipEventElapsedTime(float *ms, hipEvent_t a, hipEvent_t b);

#ifdef __cplusplus
/* device work (a fake kernel) queued on stream s, run by its thread in stream order */
void fake_enqueue(hipStream_t s, std::function<void()> fn);
#endif
#endif
