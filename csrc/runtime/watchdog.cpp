// Comm watchdog of the native runtime (SURVEY.md §5 failure detection: "ncclCommGetAsyncError
// polling + abort").  The reference at least fails fast on MPI errors (MPI_ERRORS_RETURN,
// MultiGPU/Diffusion3d_Baseline/Tools.c:228-234; the exit in DiffusionMPICUDA.h:62-63); a
// device-side exchange with a dead or hung peer, though, never returns an error: its
// kernels (RCCL's, or the ipc wait) spin, the stream never drains and the host blocks in
// hipStreamSynchronize.  This thread watches two signals while the engine steps:
//   * the transport's deferred error (Transport::poll_error: ncclCommGetAsyncError);
//   * the main thread's progress: Engine::steps beats after every step it enqueues, and
//     HIP blocks an enqueue once the stream's queue is full, so beats stop when the device
//     work stops.  No beat for ADVDIFF_COMM_TIMEOUT seconds (default 600, as the Python
//     path's collective timeout) = a peer stopped.
// Either way it reports, calls Transport::abort (ncclCommAbort) and ends the process with
// exit code 6 — every surviving rank, without help from a launcher.
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "runtime.hpp"

namespace advdiff::rt {

static double mono_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

double Watchdog::timeout_from_env() {
  const char* v = std::getenv("ADVDIFF_COMM_TIMEOUT");
  return v ? std::atof(v) : 600.0;
}

Watchdog::Watchdog(Transport* tr, int rank, double timeout_s, FailFn on_fail, double poll_s)
    : tr_(tr), rank_(rank), timeout_(timeout_s), poll_(poll_s), on_fail_(std::move(on_fail)) {
  last_.store(mono_s());
  if (!on_fail_) {
    on_fail_ = [this](const std::string& why) {
      std::fprintf(stderr, "[watchdog] rank %d: %s: aborting the %s transport\n", rank_,
                   why.c_str(), tr_ ? tr_->name() : "?");
      std::fflush(stderr);
      if (tr_) tr_->abort();
      std::_Exit(6);
    };
  }
  if (timeout_ > 0 && tr_ != nullptr) th_ = std::thread([this] { loop(); });
}

Watchdog::~Watchdog() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void Watchdog::arm() {
  beat();
  armed_.store(true);
}

void Watchdog::disarm() { armed_.store(false); }

void Watchdog::beat() { last_.store(mono_s()); }

void Watchdog::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    cv_.wait_for(lk, std::chrono::duration<double>(poll_));
    if (stop_) break;
    const int e = tr_->poll_error();
    if (e != 0) {
      fired_ = true;
      on_fail_("transport reported asynchronous error " + std::to_string(e));
      return;
    }
    if (armed_.load() && mono_s() - last_.load() > timeout_) {
      fired_ = true;
      char b[160];
      std::snprintf(b, sizeof b, "no progress for %.0f s (ADVDIFF_COMM_TIMEOUT): a peer stopped",
                    timeout_);
      on_fail_(b);
      return;
    }
  }
}

}  // namespace advdiff::rt
