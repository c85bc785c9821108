// fnpz_guard.h — no C++ exception crosses libfednpz's C ABI.
//
// Every extern "C" entry point runs its body through guard(): an allocation that fails
// (std::bad_alloc) or a thread that cannot be created (std::system_error) is FNPZ_ENOMEM, anything
// else FNPZ_EINVAL, with the reason in fnpz_last_error() — instead of std::terminate aborting the
// combiner process. Worker threads hand their exception to the caller (FirstError), and
// pools that cannot create a thread go on with the ones they have (the caller always works too).
#pragma once

#include <algorithm>
#include <atomic>
#include <exception>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/fednpz.h"

namespace fnpz_internal {

int set_error(int code, const char* fmt, ...);

template <class F>
int guard(const char* who, F&& f) noexcept {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return set_error(FNPZ_ENOMEM, "%s: out of memory", who);
    } catch (const std::system_error& e) {
        return set_error(FNPZ_ENOMEM, "%s: %s", who, e.what());
    } catch (const std::exception& e) {
        return set_error(FNPZ_EINVAL, "%s: %s", who, e.what());
    } catch (...) {
        return set_error(FNPZ_EINVAL, "%s: unknown error", who);
    }
}

// the first exception thrown by any of a job's workers, rethrown on the calling thread
class FirstError {
   public:
    void capture() noexcept {
        std::lock_guard<std::mutex> lk(mu_);
        if (!err_) err_ = std::current_exception();
    }
    void rethrow() const {
        if (err_) std::rethrow_exception(err_);
    }

   private:
    std::mutex mu_;
    std::exception_ptr err_;
};

// f(i) for i in [0, n) on the caller and up to threads - 1 new threads (fewer if the system will
// not create them); the first exception of any of them is rethrown here once all have joined
template <class F>
void run_parallel(int n, int threads, F&& f) {
    threads = std::max(1, std::min(threads, n));
    std::atomic<int> next{0};
    FirstError err;
    auto work = [&] {
        try {
            for (int i; (i = next.fetch_add(1)) < n;) f(i);
        } catch (...) {
            err.capture();
            next.store(n);   // the others stop at their next claim
        }
    };
    std::vector<std::thread> pool;
    try {
        for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    } catch (...) {
        // no more threads (or no room to hold one): the ones started and the caller finish the job
    }
    work();
    for (auto& th : pool) th.join();
    err.rethrow();
}

}  // namespace fnpz_internal
