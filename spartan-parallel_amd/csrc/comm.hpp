// spg — the cross-rank exchange of an SPMD call (spg_set_comm / spg_set_comm_rccl), host only: shared by the
// prover (api.hip comm_allgather / comm_sum_fq, which every sharded R1CSProof / SPARK / multi_evaluate exchange
// goes through) and the CPU test library (hostcheck.cpp), so the CPU suite runs this exact code on gloo ranks.
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/spg.h"
#include "field.hpp"

namespace spg {

// allgather through fn with every rank's 8-byte status in front of its payload: recv receives rank 0's `bytes`,
// then rank 1's, ...; *first_status = the first non-zero status over the ranks in rank order (this rank's own
// `status` included), 0 when all succeeded. Returns fn's result (non-zero: the transport itself failed).
inline int allgather_with_status(spg_allgather_fn fn, void* user, int nranks, int status, const void* send,
                                 size_t bytes, std::vector<uint8_t>& recv, int64_t* first_status) {
  const size_t rec = 8 + bytes;
  std::vector<uint8_t> mine(rec, 0), all(rec * (size_t)nranks);
  const int64_t st = status;
  memcpy(mine.data(), &st, 8);
  if (bytes) memcpy(mine.data() + 8, send, bytes);
  const int rc = fn(user, mine.data(), rec, all.data());
  *first_status = 0;
  if (rc) return rc;
  recv.resize(bytes * (size_t)nranks);
  for (int q = 0; q < nranks; q++) {
    int64_t s;
    memcpy(&s, all.data() + q * rec, 8);
    if (!*first_status && s) *first_status = s;
    if (bytes) memcpy(recv.data() + q * bytes, all.data() + q * rec + 8, bytes);
  }
  return 0;
}

// out[i] = the sum mod q over the ranks of element i of their n-scalar vectors (all: rank-major, as gathered)
inline void sum_over_ranks(const uint8_t* all, int nranks, size_t n, Fq* out) {
  const Fq* a = (const Fq*)all;
  for (size_t i = 0; i < n; i++) {
    Fq acc = a[i];
    for (int q = 1; q < nranks; q++) acc = fq_add(acc, a[(size_t)q * n + i]);
    out[i] = acc;
  }
}

}  // namespace spg
