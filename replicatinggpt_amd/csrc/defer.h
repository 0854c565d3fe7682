// charpt deferred work (include/charpt.h "Deferred work"): the split-K reduces a cg_gemm call with
// CG_GEMM_DEFER_REDUCE leaves pending, the AdamW updates of cg_adamw_defer and the column-sum reduces
// of the CG_DEFER calls.  Every queue belongs to ONE stream of one device: only a persistent GEMM
// launch on that stream takes its jobs, cg_flush_deferred(stream) launches the rest, and a mutex
// guards the registry -- host threads that each drive their own stream share no state.
#pragma once
#include <mutex>

#include "gemm_common.h"

namespace cg {

// one queued column-sum reduce (reduce_partials_deferrable): outputs a / b / c, S columns each
struct PartJob {
    const float* part;
    int64_t K, N, S;
    float *a, *b, *c;
    int acc, acc_c;
};
constexpr int MAX_PART_JOBS = 24;
struct PartJobs {
    int n;
    int start[MAX_PART_JOBS + 1];   // first block of job q; start[n] = the grid
    PartJob j[MAX_PART_JOBS];
};

constexpr int MAX_ADAM_PENDING = 64;

struct DeferQueue {
    hipStream_t stream = nullptr;
    int device = -1;
    RedJob red[MAX_RED];
    int nred = 0;
    AdamJob adam[MAX_ADAM_PENDING];
    int nadam = 0;
    int adam_taken = 0;   // AdamW jobs GEMM launches took since the last flush / discard
    PartJobs parts = {};
};

// the registry lock; every function below expects the caller to hold it
std::mutex& defer_mutex();
// the queue of stream st (keyed by the stream's own device); nullptr when it has none and !create
DeferQueue* defer_queue(hipStream_t st, bool create);
// remove an emptied queue from the registry (q is invalid afterwards)
void defer_queue_drop(DeferQueue* q);
// queued column-sum reduces whose outputs overlap [p, p + n) go out now (util.hip)
void flush_parts_touching_locked(DeferQueue* q, const float* p, int64_t n);
// launch (on the queue's stream) and clear one kind of job
void flush_red_locked(DeferQueue& q);
void flush_adam_locked(DeferQueue& q);
void flush_parts_locked(DeferQueue& q);   // util.hip

}  // namespace cg
