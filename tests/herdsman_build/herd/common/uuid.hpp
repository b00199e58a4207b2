// Test-only include shim: herdsman's i_worker_group.hpp includes this header
// from the (empty) herd_common submodule; it maps to the backend's stand-in
// task types (herdsman_amd/host/herd_common_standin.hpp).
#pragma once
#include "herd_common_standin.hpp"
