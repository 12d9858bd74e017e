// Tracker <-> mapper state exchange on the device.
//
// Replaces the reference's ShareData (src/share.py:27-166) served by a
// multiprocessing BaseManager (voxslam.py:28-33): there every
// update_share_data (mapping.py:236-248) deep-copies the decoder and each
// map_states tensor to the host, pickles them into the manager process, and
// every do_tracking (tracking.py:114-125) pickles them back out and re-uploads
// them with .cuda().  Here the state never leaves HBM:
//
//   * a POSIX shared-memory control block (one per ShareData) holds a robust
//     process-shared mutex, the stop flags, the tracked trajectory and, per
//     channel (decoder / points_encoder / states / ...), three slots;
//   * a slot is a device allocation owned by the publishing process and
//     exported once per (re)allocation with hipIpcGetMemHandle;
//   * publish = D2D copies of the writer's tensors into a slot nobody reads
//     (never the latest one), one stream sync, then the slot becomes `latest`
//     under the mutex — readers never see a half-written snapshot and the
//     writer never waits for a reader (3 slots: latest, one held by a reader,
//     one free);
//   * fetch = pin the latest slot (reader count), open its IPC handle (cached
//     per slot generation), D2D copies into the reader's own buffers, unpin.
//
// The reference's deepcopy semantics hold: the reader owns private copies.
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime.h>

#include "psvo_common.h"

namespace {

constexpr uint32_t kMagic = 0x50535631u;  // "PSV1"
constexpr int kSlots = 3;
constexpr int64_t kAlign = 256;

struct Slot {
    uint64_t version;      // 0 = never published
    uint32_t generation;   // bumped when the writer reallocates the region
    int32_t readers;       // pinned by fetches in flight
    int32_t writing;       // a publish is filling it
    int32_t device;
    int32_t owner_pid;
    int32_t pad;
    uint64_t owner_ptr;    // the writer's own pointer (same-process fetches)
    int64_t capacity;
    int64_t used;
    hipIpcMemHandle_t handle;
    int64_t meta_len;
    char meta[PSVO_SHARE_META_CAP];
};

struct Channel {
    int32_t latest;        // slot index of the newest snapshot, -1 = none
    int32_t writer_pid;
    uint64_t next_version;
    Slot slot[kSlots];
};

struct Block {
    uint32_t magic;
    uint32_t size;
    pthread_mutex_t mu;
    int32_t flags[PSVO_SHARE_FLAGS];
    int64_t traj_count;
    double traj[PSVO_SHARE_TRAJ_CAP][PSVO_SHARE_POSE_DIM];
    Channel ch[PSVO_SHARE_CHANNELS];
};

struct Handle {
    Block *b;
    char name[128];
    bool owner;                                        // created the segment
    // writer side: this process's allocation behind each slot
    void *own_ptr[PSVO_SHARE_CHANNELS][kSlots];
    int64_t own_cap[PSVO_SHARE_CHANNELS][kSlots];
    uint32_t own_gen[PSVO_SHARE_CHANNELS][kSlots];
    // reader side: the mapping opened for each slot generation
    void *map_ptr[PSVO_SHARE_CHANNELS][kSlots];
    uint32_t map_gen[PSVO_SHARE_CHANNELS][kSlots];
};

using psvo::set_error;

int lock(Block *b) {
    int rc = pthread_mutex_lock(&b->mu);
    if (rc == EOWNERDEAD) {  // a process died holding it: the block stays consistent (single-word updates)
        pthread_mutex_consistent(&b->mu);
        rc = 0;
    }
    return rc;
}

void unlock(Block *b) { pthread_mutex_unlock(&b->mu); }

struct Guard {
    Block *b;
    int rc;
    explicit Guard(Block *b_) : b(b_), rc(lock(b_)) {}
    ~Guard() {
        if (rc == 0) unlock(b);
    }
};

double now_ms() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

Handle *map_block(const char *name, bool create) {
    const int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) {
        set_error(PSVO_E_SYSTEM, "shm_open(%s): %s", name, strerror(errno));
        return nullptr;
    }
    if (create && ftruncate(fd, sizeof(Block)) != 0) {
        set_error(PSVO_E_SYSTEM, "ftruncate(%s): %s", name, strerror(errno));
        close(fd);
        shm_unlink(name);
        return nullptr;
    }
    void *p = mmap(nullptr, sizeof(Block), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        set_error(PSVO_E_SYSTEM, "mmap(%s): %s", name, strerror(errno));
        if (create) shm_unlink(name);
        return nullptr;
    }
    Block *b = static_cast<Block *>(p);
    if (create) {
        memset(b, 0, sizeof(Block));
        pthread_mutexattr_t at;
        pthread_mutexattr_init(&at);
        pthread_mutexattr_setpshared(&at, PTHREAD_PROCESS_SHARED);
        pthread_mutexattr_setrobust(&at, PTHREAD_MUTEX_ROBUST);
        pthread_mutex_init(&b->mu, &at);
        pthread_mutexattr_destroy(&at);
        for (int c = 0; c < PSVO_SHARE_CHANNELS; ++c) b->ch[c].latest = -1;
        b->size = sizeof(Block);
        __atomic_store_n(&b->magic, kMagic, __ATOMIC_RELEASE);
    } else if (__atomic_load_n(&b->magic, __ATOMIC_ACQUIRE) != kMagic || b->size != sizeof(Block)) {
        munmap(p, sizeof(Block));
        set_error(PSVO_E_SYSTEM, "shm segment %s is not a psvo share block of this build", name);
        return nullptr;
    }
    Handle *h = new Handle();
    memset(h, 0, sizeof(Handle));
    h->b = b;
    snprintf(h->name, sizeof(h->name), "%s", name);
    h->owner = create;
    return h;
}

}  // namespace

extern "C" {

int64_t psvo_share_block_bytes(void) { return (int64_t)sizeof(Block); }

void *psvo_share_create(const char *name) {
    if (!name || name[0] != '/' || strlen(name) >= 128) {
        set_error(PSVO_E_INVALID, "share name must start with '/' and be < 128 chars");
        return nullptr;
    }
    return map_block(name, true);
}

void *psvo_share_attach(const char *name) {
    if (!name || name[0] != '/' || strlen(name) >= 128) {
        set_error(PSVO_E_INVALID, "share name must start with '/' and be < 128 chars");
        return nullptr;
    }
    return map_block(name, false);
}

void psvo_share_detach(void *handle) {
    Handle *h = static_cast<Handle *>(handle);
    if (!h) return;
    for (int c = 0; c < PSVO_SHARE_CHANNELS; ++c)
        for (int s = 0; s < kSlots; ++s) {
            if (h->map_ptr[c][s]) (void)hipIpcCloseMemHandle(h->map_ptr[c][s]);
            if (h->own_ptr[c][s]) (void)hipFree(h->own_ptr[c][s]);
        }
    munmap(h->b, sizeof(Block));
    delete h;
}

int psvo_share_unlink(const char *name) {
    if (shm_unlink(name) != 0 && errno != ENOENT) return set_error(PSVO_E_SYSTEM, "shm_unlink(%s): %s", name, strerror(errno));
    return PSVO_OK;
}

int psvo_share_set_flag(void *handle, int i, int value) {
    Handle *h = static_cast<Handle *>(handle);
    PSVO_REQUIRE(h && i >= 0 && i < PSVO_SHARE_FLAGS, "share_set_flag: bad handle / flag %d", i);
    __atomic_store_n(&h->b->flags[i], value, __ATOMIC_SEQ_CST);
    return PSVO_OK;
}

int psvo_share_get_flag(void *handle, int i) {
    Handle *h = static_cast<Handle *>(handle);
    if (!h || i < 0 || i >= PSVO_SHARE_FLAGS) return -1;
    return __atomic_load_n(&h->b->flags[i], __ATOMIC_SEQ_CST);
}

int psvo_share_push_pose(void *handle, const double *pose, int n) {
    Handle *h = static_cast<Handle *>(handle);
    PSVO_REQUIRE(h && pose && n > 0 && n < PSVO_SHARE_POSE_DIM, "share_push_pose: bad arguments (n=%d)", n);
    Guard g(h->b);
    PSVO_REQUIRE(g.rc == 0, "share_push_pose: mutex error %d", g.rc);
    PSVO_REQUIRE(h->b->traj_count < PSVO_SHARE_TRAJ_CAP, "share_push_pose: trajectory full (%d poses)",
                 PSVO_SHARE_TRAJ_CAP);
    double *row = h->b->traj[h->b->traj_count];
    row[0] = n;  // row = [n, pose[0..n), 0...]
    for (int k = 1; k < PSVO_SHARE_POSE_DIM; ++k) row[k] = k <= n ? pose[k - 1] : 0.0;
    h->b->traj_count++;
    return PSVO_OK;
}

int64_t psvo_share_trajectory(void *handle, double *out, int64_t cap) {
    Handle *h = static_cast<Handle *>(handle);
    if (!h) return -1;
    Guard g(h->b);
    if (g.rc != 0) return -1;
    const int64_t n = h->b->traj_count;
    if (out) memcpy(out, h->b->traj, sizeof(double) * PSVO_SHARE_POSE_DIM * (n < cap ? n : cap));
    return n;
}

// Writer: copy `n` device buffers into a free slot of `channel` (at 256-B
// aligned offsets, written to `offsets`) and make it the latest snapshot.
int psvo_share_publish(void *handle, void *stream, int channel, int n, const void *const *srcs, const int64_t *bytes,
                       const void *meta, int64_t meta_len, int timeout_ms, int64_t *offsets, uint64_t *version) {
    Handle *h = static_cast<Handle *>(handle);
    PSVO_REQUIRE(h && channel >= 0 && channel < PSVO_SHARE_CHANNELS, "share_publish: bad handle / channel %d",
                 channel);
    PSVO_REQUIRE(n >= 0 && (n == 0 || (srcs && bytes && offsets)), "share_publish: bad buffer list");
    PSVO_REQUIRE(meta_len >= 0 && meta_len <= PSVO_SHARE_META_CAP, "share_publish: meta of %lld B exceeds %d B",
                 (long long)meta_len, PSVO_SHARE_META_CAP);
    int64_t need = 0;
    for (int i = 0; i < n; ++i) {
        PSVO_REQUIRE(bytes[i] >= 0 && (bytes[i] == 0 || srcs[i]), "share_publish: buffer %d invalid", i);
        offsets[i] = need;
        need += (bytes[i] + kAlign - 1) / kAlign * kAlign;
    }
    Block *b = h->b;
    Channel &ch = b->ch[channel];
    const int pid = (int)getpid();
    // 1. claim a slot that is neither the latest nor pinned by a reader
    int s = -1;
    const double t0 = now_ms();
    for (;;) {
        {
            Guard g(b);
            PSVO_REQUIRE(g.rc == 0, "share_publish: mutex error %d", g.rc);
            PSVO_REQUIRE(ch.writer_pid == 0 || ch.writer_pid == pid,
                         "share_publish: channel %d already has a writer (pid %d)", channel, ch.writer_pid);
            ch.writer_pid = pid;
            uint64_t best = ~0ull;
            for (int k = 0; k < kSlots; ++k) {
                const Slot &sl = ch.slot[k];
                if (k == ch.latest || sl.readers > 0 || sl.writing) continue;
                if (sl.version < best) best = sl.version, s = k;
            }
            if (s >= 0) ch.slot[s].writing = 1;
        }
        if (s >= 0) break;
        if (now_ms() - t0 > timeout_ms) return set_error(PSVO_E_BUSY, "share_publish: no free slot in %d ms", timeout_ms);
        usleep(50);
    }
    Slot &sl = ch.slot[s];
    auto fail = [&](int code, const char *what, hipError_t e) {
        Guard g(b);
        sl.writing = 0;
        return set_error(code, "share_publish: %s: %s", what, hipGetErrorString(e));
    };
    // 2. (re)allocate this process's region behind the slot, export it once
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail(PSVO_E_LAUNCH, "hipGetDevice", e);
    const int64_t alloc = need > 0 ? need : kAlign;
    if (!h->own_ptr[channel][s] || h->own_cap[channel][s] < alloc) {
        if (h->own_ptr[channel][s]) (void)hipFree(h->own_ptr[channel][s]);
        h->own_ptr[channel][s] = nullptr;
        const int64_t cap = alloc + alloc / 2;  // headroom: the map grows frame by frame
        void *p = nullptr;
        e = hipMalloc(&p, cap);
        if (e != hipSuccess) return fail(PSVO_E_LAUNCH, "hipMalloc", e);
        hipIpcMemHandle_t ipc;
        e = hipIpcGetMemHandle(&ipc, p);
        if (e != hipSuccess) {
            (void)hipFree(p);
            return fail(PSVO_E_LAUNCH, "hipIpcGetMemHandle", e);
        }
        h->own_ptr[channel][s] = p;
        h->own_cap[channel][s] = cap;
        h->own_gen[channel][s] = sl.generation + 1;
        Guard g(b);
        sl.handle = ipc;
        sl.capacity = cap;
        sl.generation = h->own_gen[channel][s];
        sl.owner_ptr = (uint64_t)(uintptr_t)p;
        sl.owner_pid = pid;
        sl.device = dev;
    }
    // 3. fill it and wait for the copies (readers may be other processes)
    hipStream_t st = psvo::as_stream(stream);
    char *base = static_cast<char *>(h->own_ptr[channel][s]);
    for (int i = 0; i < n; ++i) {
        if (bytes[i] == 0) continue;
        e = hipMemcpyAsync(base + offsets[i], srcs[i], bytes[i], hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return fail(PSVO_E_LAUNCH, "hipMemcpyAsync", e);
    }
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(PSVO_E_LAUNCH, "hipStreamSynchronize", e);
    // 4. publish
    Guard g(b);
    PSVO_REQUIRE(g.rc == 0, "share_publish: mutex error %d", g.rc);
    sl.used = need;
    sl.meta_len = meta_len;
    if (meta_len) memcpy(sl.meta, meta, meta_len);
    sl.version = ++ch.next_version;
    sl.writing = 0;
    ch.latest = s;
    if (version) *version = sl.version;
    return PSVO_OK;
}

// Reader: pin the latest snapshot of `channel` if its version is > `after`.
// Returns 1 (pinned: *slot, *version, meta and *base filled), 0 (nothing
// newer) or a negative error (-code; psvo_last_error()).
int psvo_share_acquire(void *handle, int channel, uint64_t after, int *slot, uint64_t *version, void *meta,
                       int64_t meta_cap, int64_t *meta_len, int64_t *used, void **base) {
    Handle *h = static_cast<Handle *>(handle);
    if (!h || channel < 0 || channel >= PSVO_SHARE_CHANNELS || !slot || !version || !base)
        return -set_error(PSVO_E_INVALID, "share_acquire: bad arguments");
    Block *b = h->b;
    Channel &ch = b->ch[channel];
    int s;
    uint32_t gen;
    int owner;
    uint64_t owner_ptr;
    hipIpcMemHandle_t ipc;
    {
        Guard g(b);
        if (g.rc != 0) return -set_error(PSVO_E_SYSTEM, "share_acquire: mutex error %d", g.rc);
        s = ch.latest;
        if (s < 0 || ch.slot[s].version <= after) return 0;
        Slot &sl = ch.slot[s];
        if (meta_len) *meta_len = sl.meta_len;
        if (sl.meta_len > meta_cap && meta) return -set_error(PSVO_E_INVALID, "share_acquire: meta buffer too small");
        if (meta && sl.meta_len) memcpy(meta, sl.meta, sl.meta_len);
        if (used) *used = sl.used;
        sl.readers++;
        *version = sl.version;
        gen = sl.generation;
        owner = sl.owner_pid;
        owner_ptr = sl.owner_ptr;
        ipc = sl.handle;
    }
    *slot = s;
    if (owner == (int)getpid()) {  // same process: the writer's pointer (IPC cannot reopen its own memory)
        *base = (void *)(uintptr_t)owner_ptr;
        return 1;
    }
    if (!h->map_ptr[channel][s] || h->map_gen[channel][s] != gen) {
        if (h->map_ptr[channel][s]) (void)hipIpcCloseMemHandle(h->map_ptr[channel][s]);
        h->map_ptr[channel][s] = nullptr;
        void *p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, ipc, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            Guard g(b);
            ch.slot[s].readers--;
            return -set_error(PSVO_E_LAUNCH, "share_acquire: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
        }
        h->map_ptr[channel][s] = p;
        h->map_gen[channel][s] = gen;
    }
    *base = h->map_ptr[channel][s];
    return 1;
}

// Reader: D2D copies out of a pinned slot, then wait for them.
int psvo_share_read(void *handle, void *stream, int channel, int slot, int n, void *const *dsts,
                    const int64_t *offsets, const int64_t *bytes, const void *base) {
    Handle *h = static_cast<Handle *>(handle);
    PSVO_REQUIRE(h && channel >= 0 && channel < PSVO_SHARE_CHANNELS && slot >= 0 && slot < kSlots && base,
                 "share_read: bad arguments");
    const int64_t used = h->b->ch[channel].slot[slot].used;
    hipStream_t st = psvo::as_stream(stream);
    for (int i = 0; i < n; ++i) {
        if (bytes[i] == 0) continue;
        PSVO_REQUIRE(dsts[i] && offsets[i] >= 0 && offsets[i] + bytes[i] <= used,
                     "share_read: buffer %d [%lld, +%lld) outside the snapshot (%lld B)", i, (long long)offsets[i],
                     (long long)bytes[i], (long long)used);
        const hipError_t e = hipMemcpyAsync(dsts[i], static_cast<const char *>(base) + offsets[i], bytes[i],
                                            hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return set_error(PSVO_E_LAUNCH, "share_read: hipMemcpyAsync: %s", hipGetErrorString(e));
    }
    const hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return set_error(PSVO_E_LAUNCH, "share_read: hipStreamSynchronize: %s", hipGetErrorString(e));
    return PSVO_OK;
}

int psvo_share_release(void *handle, int channel, int slot) {
    Handle *h = static_cast<Handle *>(handle);
    PSVO_REQUIRE(h && channel >= 0 && channel < PSVO_SHARE_CHANNELS && slot >= 0 && slot < kSlots,
                 "share_release: bad arguments");
    Guard g(h->b);
    PSVO_REQUIRE(g.rc == 0, "share_release: mutex error %d", g.rc);
    Slot &sl = h->b->ch[channel].slot[slot];
    PSVO_REQUIRE(sl.readers > 0, "share_release: slot %d of channel %d is not pinned", slot, channel);
    sl.readers--;
    return PSVO_OK;
}

uint64_t psvo_share_version(void *handle, int channel) {
    Handle *h = static_cast<Handle *>(handle);
    if (!h || channel < 0 || channel >= PSVO_SHARE_CHANNELS) return 0;
    Guard g(h->b);
    const int s = h->b->ch[channel].latest;
    return s < 0 ? 0 : h->b->ch[channel].slot[s].version;
}

}  // extern "C"
