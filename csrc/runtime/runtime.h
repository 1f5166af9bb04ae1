// pytorch_r2d2_amd host runtime (C++17, C ABI; loaded with ctypes).
//
//  * sumtree   -- 64-ary sum tree over doubles: batched leaf updates, stratified proportional
//                 sampling in O(B log64 N).  Host twin of the HBM tree in csrc/kernels/replay.hip
//                 (used by the host ReplayMemory and the CPU learner path).
//  * ring      -- single-producer / single-consumer byte ring in POSIX shared memory with
//                 acquire/release head/tail counters: the actor -> learner trajectory transport
//                 for CPU actor processes (replaces the reference's pickle files guarded by
//                 fasteners locks, replay_memory.py:125-173).
//  * lock      -- fcntl advisory locks on a dedicated lock file (the reference uses the data file
//                 itself as its lock).
//  * heartbeat -- shared-memory table of per-process heartbeats for the supervisor / watchdog.
#pragma once
#include <stdint.h>

extern "C" {
// sum tree
void* r2rt_sumtree_create(int64_t capacity);
void r2rt_sumtree_destroy(void* t);
int64_t r2rt_sumtree_capacity(void* t);
void r2rt_sumtree_set(void* t, const int64_t* idx, const double* val, int64_t n);
void r2rt_sumtree_rebuild(void* t, const double* leaves);
double r2rt_sumtree_total(void* t);
double r2rt_sumtree_get(void* t, int64_t idx);
void r2rt_sumtree_sample(void* t, const double* u01, int64_t n, int stratified, int64_t* out_idx,
                         double* out_p);

// SPSC shared-memory ring
void* r2rt_ring_open(const char* name, uint64_t capacity, int create);
int r2rt_ring_push(void* r, const void* data, uint32_t len);
int64_t r2rt_ring_pop(void* r, void* out, uint32_t maxlen);
int64_t r2rt_ring_peek(void* r);
// zero-copy consumer: pointer to the front record's payload (valid until r2rt_ring_release)
int64_t r2rt_ring_front(void* r, const void** payload);
void r2rt_ring_release(void* r);
void* r2rt_ring_mapping(void* r, uint64_t* len);
uint64_t r2rt_ring_used(void* r);
uint64_t r2rt_ring_capacity(void* r);
void r2rt_ring_close(void* r, int unlink);

// fcntl lock
int r2rt_lock_open(const char* path);
int r2rt_lock_acquire(int fd, int blocking);
int r2rt_lock_release(int fd);
void r2rt_lock_close(int fd);

// heartbeat table
void* r2rt_hb_open(const char* name, int n_slots, int create);
void r2rt_hb_beat(void* h, int slot, uint64_t counter, int32_t status);
int r2rt_hb_read(void* h, int slot, uint64_t* last_ns, uint64_t* counter, int32_t* pid,
                 int32_t* status);
uint64_t r2rt_now_ns();
void r2rt_hb_close(void* h, int unlink);

int r2rt_version();

// versioned single-writer / many-reader blob in shared memory (seqlock): weight publication
// from the learner process to CPU actor processes
void* r2rt_slot_open(const char* name, uint64_t bytes, int create);
void r2rt_slot_write(void* s, const void* data, uint64_t bytes, int64_t version);
// 1 = copied a version newer than `have`, 0 = nothing newer, -1 = torn after retries
int r2rt_slot_read(void* s, void* out, uint64_t bytes, int64_t have, int64_t* version);
int64_t r2rt_slot_version(void* s);
void r2rt_slot_close(void* s, int unlink);
}
