// pinned.h — host staging for polled matches: pinned (page-locked) memory, grown on demand and reused
// across polls, so the device->host copies of sg_poll_matches / sg_get_projection run at the DMA rate
// instead of through pageable bounce buffers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <new>

template <class T> struct PinnedVec {
    T* p = nullptr;
    size_t cap = 0;
    PinnedVec() = default;
    PinnedVec(const PinnedVec&) = delete;
    PinnedVec& operator=(const PinnedVec&) = delete;
    ~PinnedVec() {
        if (p) (void)hipHostFree(p);
    }
    // room for n elements (contents are not kept when it grows)
    void resize(size_t n) {
        if (n <= cap) return;
        size_t c = cap ? cap : 1024;
        while (c < n) c *= 2;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault) != hipSuccess) throw std::bad_alloc();
        cap = c;
    }
    T* data() { return p; }
};
