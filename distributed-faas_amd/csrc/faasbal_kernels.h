// faasbal_kernels.h -- internal: constants and kernel argument blocks.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace fb {

constexpr int kBS = 256;           // threads per workgroup (4 wave64)
constexpr int kWaves = kBS / 64;
constexpr int kFItems = 8;         // log entries per thread in log-role blocks
constexpr int kFTile = kBS * kFItems;
constexpr int kRsItems = 8;        // radix sort: keys per thread per tile
constexpr int kRsTile = kBS * kRsItems;

// event kinds / status (include/faasbal.h)
constexpr int kEvRegister = 0, kEvReconnect = 1, kEvHeartbeat = 2, kEvResult = 3;
constexpr uint8_t kEvsApplied = 0, kEvsReconnect = 1;

// per-slot tick status (st)
constexpr uint8_t kStAlive = 1;      // registered and alive after the final purge
constexpr uint8_t kStDiedStart = 2;  // the registration alive at tick start died this tick
constexpr uint8_t kStEvicted = 4;    // record deleted during the tick and not re-created
// post_flags: bit0 died_start, bits 1-2 queue status after the tick's messages
constexpr int kPfDiedStart = 1;
constexpr int kQsKeep = 0, kQsOut = 1, kQsFront = 2, kQsBack = 3;

// device-resident per-tick scalars (zeroed by every launch)
struct DevParams {
    unsigned long long cap_total;  // sum of c over live queued workers
    unsigned long long new_qlen;   // next LRU queue length
    int64_t O;                     // orphans
    int64_t n_evicted;
    int64_t N_eff;                 // tasks dispatched
    int64_t p;                     // tasks of the partial round L
    int64_t AL;                    // |A_L|
    int32_t maxc;                  // max c
    int32_t L;                     // fill level
    int32_t status;                // 1 = round table too narrow (rerun wider), 2 = log full
    int32_t pad;
};

struct EvArgs {
    int E;
    uint32_t tick;
    double tte;
    int64_t head_in;
    const uint32_t *skeys, *svals;
    const uint8_t *ev_kind;
    const int32_t *ev_val;
    const double *ev_ts;
    const int64_t *ev_seq;
    uint8_t *ev_status;
    const uint8_t *reg;
    const int32_t *free_in;
    const double *hb;
    const uint32_t *epoch;
    const uint8_t *inq_in;
    int32_t *log_slot;
    uint8_t *post_reg;
    int32_t *post_free;
    double *post_hb;
    uint32_t *post_epoch;
    uint8_t *post_flags;
    uint32_t *touched;
    int32_t *front_list, *back_list;
};

struct SlotArgs {
    int W;
    uint32_t tick;
    double now, tte;
    const uint32_t *touched;
    const uint8_t *reg;
    const double *hb;
    const int32_t *free_in;
    const uint8_t *post_reg;
    const double *post_hb;
    const int32_t *post_free;
    const uint8_t *post_flags;
    uint8_t *st;
    int32_t *free_out;
    uint8_t *inq_out;
    uint32_t *wcnt;
};

struct ScanArgs {
    int nbf, nbq, R, E;
    uint32_t tick;
    int64_t Qn, Qlog, head_in, log_lo;
    const int32_t *log_slot;
    const uint8_t *st;
    const uint32_t *epoch;
    const uint32_t *touched;
    const uint8_t *post_flags;
    const int32_t *front_list, *queue_in, *back_list;
    const int32_t *free_out;
    int32_t *c_arr;
    uint32_t *fcnt;
    uint32_t *qcnt;
    int32_t *qbmax;
    DevParams *P;
};

struct PlanArgs {
    int nbf, nbw, nbq, R;
    const uint32_t *fcnt, *wcnt, *qcnt;
    const int32_t *qbmax;
    int64_t *fpre, *wpre, *qpre, *A;
    DevParams *P;
};

struct EmitArgs {
    int nbq, nbf, W, R, E;
    int64_t Qn, Qlog, head_in, log_lo, T, log_cap;
    const int32_t *c_arr;
    const int32_t *front_list, *queue_in, *back_list;
    const int64_t *qpre, *A, *fpre, *wpre;
    const int32_t *qbmax;
    const uint8_t *st;
    const uint32_t *epoch;
    const int32_t *log_slot_ro;
    int32_t *log_slot;
    int32_t *free_out;
    int32_t *queue_out;
    uint8_t *inq_out;
    int64_t *orphans;
    int32_t *evicted;
    DevParams *P;
};

struct CommitArgs {
    int W;
    uint32_t tick;
    const uint8_t *st;
    const uint32_t *touched;
    const double *post_hb;
    const uint32_t *post_epoch;
    uint8_t *reg;
    double *hb;
    uint32_t *epoch;
};

// Host-side launchers (defined in faasbal_kernels.hip; grid sizes are the caller's).
using Stream = hipStream_t;
void launch_rs_hist(const uint32_t *keys, int n, int shift, uint32_t *hist, int nblk, Stream st);
void launch_scan_1wg(uint32_t *a, int n, Stream st);
void launch_rs_scatter(const uint32_t *kin, const uint32_t *vin, uint32_t *kout, uint32_t *vout, int n,
                       int shift, const uint32_t *hist, int nblk, int identity_vals, Stream st);
void launch_ev_apply(const EvArgs &a, Stream st);
void launch_slots(const SlotArgs &a, int grid, Stream st);
void launch_scan(const ScanArgs &a, int grid, Stream st);
void launch_plan(const PlanArgs &a, int grid, Stream st);
void launch_emit(const EmitArgs &a, int grid, Stream st);
void launch_commit(const CommitArgs &a, int grid, Stream st);

}  // namespace fb
