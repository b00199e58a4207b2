// Test-only include shim for herd_common's task types (see ../../../uuid.hpp).
#pragma once
#include "herd_common_standin.hpp"
