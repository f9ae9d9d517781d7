// join_gpu_stubs.cpp -- the device entry points ewal_join.cpp's multi-context
// driver and ewal_host.cpp's directory calls use (defined by
// etcd_amd/csrc/ewal_api.hip, which only hipcc builds), answering as the
// product library does without a GPU:
// EWAL_E_NODEVICE.  Linked only into the host sanitizer build of the join
// (tests/sanitize/san_join.cpp), which never reaches them.
#include "ewal.h"

extern "C" {
int ewal_readall_range_device(ewal_ctx *, const void *, uint64_t, uint64_t, uint32_t, ewal_result *) {
  return EWAL_E_NODEVICE;
}
int ewal_copy_range_info(ewal_ctx *, ewal_range_info *) { return EWAL_E_NODEVICE; }
int64_t ewal_copy_entries(ewal_ctx *, ewal_entry *, int64_t) { return EWAL_E_NODEVICE; }
int64_t ewal_copy_split_bytes(ewal_ctx *, uint8_t *, int64_t) { return EWAL_E_NODEVICE; }
int64_t ewal_copy_unrec(ewal_ctx *, ewal_unrec *, int64_t) { return EWAL_E_NODEVICE; }
int64_t ewal_copy_unrec_bytes(ewal_ctx *, uint8_t *, int64_t) { return EWAL_E_NODEVICE; }
int ewal_download(ewal_ctx *, void *, const void *, uint64_t) { return EWAL_E_NODEVICE; }
int ewal_stage_to_device(ewal_ctx *, const void *, uint64_t, void **) { return EWAL_E_NODEVICE; }
int ewal_range_probe(ewal_ctx *, const void *, uint64_t, uint64_t, uint64_t, int64_t *, int64_t *) {
  return EWAL_E_NODEVICE;
}
int ewal_range_probe_aligned(ewal_ctx *, const void *, uint64_t, uint64_t, uint64_t, uint32_t, int64_t *, int64_t *) {
  return EWAL_E_NODEVICE;
}
int ewal_stage_begin(ewal_ctx *, uint64_t) { return EWAL_E_NODEVICE; }
int ewal_stage_put(ewal_ctx *, uint64_t, const void *, uint64_t) { return EWAL_E_NODEVICE; }
int ewal_stage_readall(ewal_ctx *, uint64_t, uint64_t, ewal_result *) { return EWAL_E_NODEVICE; }
int ewal_stage_sync(ewal_ctx *) { return EWAL_E_NODEVICE; }
int esnap_verify_packed(ewal_ctx *, const void *, uint64_t, const uint64_t *, const uint64_t *, uint32_t, uint32_t,
                        int32_t *, uint32_t *, uint32_t *) {
  return EWAL_E_NODEVICE;
}
int esnap_copy_snapshot(ewal_ctx *, uint32_t, esnap_snapshot *) { return EWAL_E_NODEVICE; }
}
