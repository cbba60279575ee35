// The C++ mirror's persistent helper threads (PubKeyUtils.cpp owns the pool):
// parallel loops for the batch entry points (hashing, CPU-path batches, the
// tx-set pre-pass and checkers).
#pragma once

#include <cstddef>
#include <functional>

namespace stellar {

// Runs range(begin, end) over [0, n) in contiguous pieces on the pool (the
// calling thread takes part), serially when n < 2 * grain.
void hostParallelFor(size_t n, size_t grain, std::function<void(size_t, size_t)> const& range);
// Threads a hostParallelFor can use at once (the pool's helpers and the caller).
size_t hostPoolThreads();

}  // namespace stellar
