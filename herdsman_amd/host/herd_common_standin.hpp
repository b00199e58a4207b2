// herd_common_standin.hpp -- stand-in for the herd_common task types.
//
// herdsman's IWorkerGroup seam (/root/reference/include/execution/worker/
// i_worker_group.hpp:8-9) includes "herd/common/model/worker/task.hpp" and
// "herd/common/uuid.hpp" from the `common` submodule, which is EMPTY in the
// reference snapshot.  The types below restate what herdsman's
// own sources show of them, nothing more:
//   * MapTask / ReduceTask are aggregates built positionally as
//     {session_uuid, input ptr(s), output ptr, crypto key ptr, circuit}
//     (/root/reference/src/service/execution_service.cpp:465-471, 506-512);
//   * member names session_uuid, output_data_frame_ptr.uuid / .partition and
//     UUID::as_string() are used by lambda_http_worker_group.cpp:69-72, 96-99;
//   * InputDataFramePtr is {DataFramePtr{uuid, partition}, row_count}
//     (execution_service.cpp:448-454, 487-493);
//   * SchemaType is an enum (key_service.cpp:28 casts it to its underlying type).
// The names of the members that herdsman never spells out (InputDataFramePtr's
// pointer/row_count, CryptoKeyPtr's schema_type, the circuit) are this
// backend's choice.  herd_common's Circuit is unknown, so the stand-in circuit
// is the backend's own stack program over the ciphertexts of a row
// (INTEGRATION.md §2); the adaptor lowers a circuit through
// herdsman_gpu::lower_circuit (gpu_worker_group.cpp).
//
// Used by the stand-alone build (herd_seam.hpp without HERDSMAN_REAL_SEAM) and,
// through tests/herdsman_build/herd/common/..., by the test that compiles the
// adaptor against herdsman's real IWorkerGroup header and i_worker_group.cpp.
#pragma once
#include <cstdint>
#include <string>
#include <variant>
#include <vector>

namespace herd::common {

struct UUID {
  std::string value;
  const std::string &as_string() const { return value; }
};

enum class SchemaType : int32_t { CKKS = 0, BFV = 1 };

struct DataFramePtr {
  UUID uuid;
  uint32_t partition = 0;
};

struct InputDataFramePtr {
  DataFramePtr pointer;
  uint64_t row_count = 0;
};

struct CryptoKeyPtr {
  SchemaType schema_type = SchemaType::CKKS;
};

// Stand-in circuit: a stack program over the ciphertexts of one row.
// CKKS operands may sit at different levels: binary ops run at the lower one
// (the other operand's extra limbs dropped), RESCALE drops one level.
// ROTSUM replaces the top with sum_{i in arg} rot_i(top), arg a bit mask
// of step counts 0..30 (bit 0: the ciphertext itself), double-hoisted (one
// ModUp of c1 and one ModDown for all of them: a baby-step block of a linear
// transform).
enum class CtOp : uint32_t { PUSH_INPUT = 0, ADD = 1, SUB = 2, MUL_RELIN = 3, ROTATE = 4, RESCALE = 5, ROTSUM = 6 };
struct CircuitInstr {
  CtOp op;
  int32_t arg = 0;  // PUSH_INPUT: index of the ciphertext in the row; ROTATE: steps; ROTSUM: step mask
};
struct Circuit {
  std::vector<CircuitInstr> program;
};

struct MapTask {
  UUID session_uuid;
  InputDataFramePtr input_data_frame_ptr;
  DataFramePtr output_data_frame_ptr;
  CryptoKeyPtr crypto_key_ptr;
  Circuit circuit;
};

struct ReduceTask {
  UUID session_uuid;
  std::vector<InputDataFramePtr> input_data_frame_ptrs;
  DataFramePtr output_data_frame_ptr;
  CryptoKeyPtr crypto_key_ptr;
  Circuit circuit;
};

using task_t = std::variant<std::monostate, MapTask, ReduceTask>;

}  // namespace herd::common
