// Host buffers of the set-up path backed by transparent huge pages.
//
// A fresh 216 MB std::vector<double> costs 54 ms of 4 KiB page faults on the
// MI355X hosts (THP in "madvise" mode), 13 ms with MADV_HUGEPAGE
// (profiles/r01/host_alloc_probe.txt). The row offsets a handle keeps for
// planning and the set-up's per-row host arrays are that size at 300^3.
#pragma once

#include <sys/mman.h>

#include <cstddef>
#include <cstdlib>
#include <new>
#include <vector>

namespace aijhip {

constexpr size_t kHugeAllocMin = size_t(4) << 20;  // smaller blocks: malloc

template <class T>
struct HugePageAllocator {
    using value_type = T;
    HugePageAllocator() = default;
    template <class U>
    HugePageAllocator(const HugePageAllocator<U> &) {}
    T *allocate(size_t n) {
        const size_t b = n * sizeof(T);
        if (b >= kHugeAllocMin) {
            void *p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (p == MAP_FAILED) throw std::bad_alloc();
            (void)madvise(p, b, MADV_HUGEPAGE);  // a hint: 4 KiB pages if refused
            return static_cast<T *>(p);
        }
        void *p = std::malloc(b ? b : 1);
        if (!p) throw std::bad_alloc();
        return static_cast<T *>(p);
    }
    void deallocate(T *p, size_t n) {
        const size_t b = n * sizeof(T);
        if (b >= kHugeAllocMin) munmap(p, b);
        else std::free(p);
    }
};

template <class T, class U>
bool operator==(const HugePageAllocator<T> &, const HugePageAllocator<U> &) { return true; }
template <class T, class U>
bool operator!=(const HugePageAllocator<T> &, const HugePageAllocator<U> &) { return false; }

template <class T>
using HostVec = std::vector<T, HugePageAllocator<T>>;

}  // namespace aijhip
