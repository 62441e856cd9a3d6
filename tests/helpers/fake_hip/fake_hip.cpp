/* The CPU stand-in of the HIP runtime (hip/hip_runtime.h next to it): test infrastructure for
   tools/sanitize.sh only. */
#include "hip/hip_runtime.h"
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

static double now_s()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

struct fake_stream {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    uint64_t queued = 0, done = 0;
    bool stop = false;
    std::thread th;
    fake_stream() : th([this] { run(); }) {}
    void run()
    {
        for (;;) {
            std::function<void()> fn;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty())
                    return;
                fn = std::move(q.front());
                q.pop_front();
            }
            fn();
            {
                std::lock_guard<std::mutex> lk(mu);
                done++;
            }
            cv.notify_all();
        }
    }
    uint64_t push(std::function<void()> fn)
    {
        std::lock_guard<std::mutex> lk(mu);
        q.push_back(std::move(fn));
        cv.notify_all();
        return ++queued;
    }
    void wait(uint64_t upto)
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done >= upto; });
    }
    ~fake_stream()
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
};

struct fake_event {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t recorded = 0, done = 0;
    double t = 0.0;
};

static fake_stream *null_stream()
{
    static fake_stream *s = new fake_stream();             /* (lives to the process's end) */
    return s;
}
static fake_stream *S(hipStream_t s) { return s ? s : null_stream(); }

void fake_enqueue(hipStream_t s, std::function<void()> fn) { S(s)->push(std::move(fn)); }

const char *hipGetErrorString(hipError_t e) { return e == hipSuccess ? "success" : "fake error"; }
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipGetDevice(int *d) { *d = 0; return hipSuccess; }
hipError_t hipSetDevice(int d) { return d == 0 ? hipSuccess : hipErrorInvalidValue; }
hipError_t hipDeviceSynchronize(void) { return hipStreamSynchronize(nullptr); }
hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t a, int dev)
{
    (void)a; (void)dev;
    *v = 256;
    return hipSuccess;
}
hipError_t hipDeviceGetStreamPriorityRange(int *lo, int *hi) { *lo = 0; *hi = -1; return hipSuccess; }
hipError_t hipMalloc(void **p, size_t n)
{
    *p = aligned_alloc(256, (n + 255) & ~(size_t)255);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void *p) { free(p); return hipSuccess; }
hipError_t hipHostMalloc(void **p, size_t n, unsigned flags) { (void)flags; return hipMalloc(p, n); }
hipError_t hipHostFree(void *p) { free(p); return hipSuccess; }
hipError_t hipMemcpy(void *dst, const void *src, size_t n, hipMemcpyKind k)
{
    (void)k;
    memcpy(dst, src, n);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind k, hipStream_t s)
{
    (void)k;
    S(s)->push([=] { memcpy(dst, src, n); });
    return hipSuccess;
}
hipError_t hipMemsetAsync(void *dst, int v, size_t n, hipStream_t s)
{
    S(s)->push([=] { memset(dst, v, n); });
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned flags)
{
    (void)flags;
    *s = new fake_stream();
    return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t *s, unsigned flags, int prio)
{
    (void)prio;
    return hipStreamCreateWithFlags(s, flags);
}
hipError_t hipExtStreamCreateWithCUMask(hipStream_t *s, uint32_t n, const uint32_t *mask)
{
    (void)n; (void)mask;
    return hipStreamCreateWithFlags(s, 0);
}
hipError_t hipStreamDestroy(hipStream_t s)
{
    if (s) {
        hipStreamSynchronize(s);
        delete s;
    }
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s)
{
    fake_stream *f = S(s);
    const uint64_t upto = f->push([] {});
    f->wait(upto);
    return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t *e) { *e = new fake_event(); return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned flags) { (void)flags; return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t e) { delete e; return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s)
{
    uint64_t g;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        g = ++e->recorded;
    }
    S(s)->push([e, g] {
        {
            std::lock_guard<std::mutex> lk(e->mu);
            if (g > e->done) {
                e->done = g;
                e->t = now_s();
            }
        }
        e->cv.notify_all();
    });
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e)
{
    std::unique_lock<std::mutex> lk(e->mu);
    const uint64_t g = e->recorded;
    e->cv.wait(lk, [&] { return e->done >= g; });
    return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e)
{
    std::lock_guard<std::mutex> lk(e->mu);
    return e->done >= e->recorded ? hipSuccess : hipErrorNotReady;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned flags)
{
    (void)flags;
    uint64_t g;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        g = e->recorded;                               /* the latest record before this call */
    }
    S(s)->push([e, g] {
        std::unique_lock<std::mutex> lk(e->mu);
        e->cv.wait(lk, [&] { return e->done >= g; });
    });
    return hipSuccess;
}
hipError_t hipEventElapsedTime(float *ms, hipEvent_t a, hipEvent_t b)
{
    std::lock_guard<std::mutex> la(a->mu);
    std::lock_guard<std::mutex> lb(b->mu);
    if (a->done < a->recorded || b->done < b->recorded || !a->recorded || !b->recorded)
        return hipErrorNotReady;
    *ms = (float)((b->t - a->t) * 1e3);
    return hipSuccess;
}
