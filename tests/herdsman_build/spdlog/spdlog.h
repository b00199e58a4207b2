// Test-only stand-in for spdlog (absent in this image): i_worker_group.cpp
// includes it without logging anything.
#pragma once
namespace spdlog {
template <class... A> void info(A &&...) {}
template <class... A> void debug(A &&...) {}
template <class... A> void warn(A &&...) {}
template <class... A> void error(A &&...) {}
}  // namespace spdlog
