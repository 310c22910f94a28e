// Peer-memory mapping for the data-parallel exchange on one node (dq_peer):
// IPC handles of the flat gradient / parameter / flag buffers, exchanged by the host
// (torch.distributed), opened by every other learner.  The exchange itself runs inside the
// backward's grouped launches (nature_cnn.hip, backward_peer).
#include <cstring>

#include "common.h"

using namespace dq;

extern "C" {

int dq_peer_ipc_get(const void* ptr, dq_ipc_handle* out) {
  DQ_CHECK_ARG(ptr && out, "null argument");
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  DQ_CHECK_HIP(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr));
  DQ_CHECK_ARG(base != nullptr, "not device memory");
  hipIpcMemHandle_t h;
  DQ_CHECK_HIP(hipIpcGetMemHandle(&h, (void*)base));
  static_assert(sizeof(h) <= sizeof(out->handle), "hipIpcMemHandle_t larger than dq_ipc_handle");
  memset(out->handle, 0, sizeof(out->handle));
  memcpy(out->handle, &h, sizeof(h));
  out->offset = (int64_t)((const char*)ptr - (const char*)base);
  return DQ_OK;
}

int dq_peer_ipc_open(const dq_ipc_handle* h, void** ptr_out, void** base_out) {
  DQ_CHECK_ARG(h && ptr_out && base_out, "null argument");
  hipIpcMemHandle_t hh;
  memcpy(&hh, h->handle, sizeof(hh));
  void* base = nullptr;
  DQ_CHECK_HIP(hipIpcOpenMemHandle(&base, hh, hipIpcMemLazyEnablePeerAccess));
  *base_out = base;
  *ptr_out = (char*)base + h->offset;
  return DQ_OK;
}

int dq_peer_ipc_close(void* base) {
  DQ_CHECK_ARG(base, "null argument");
  DQ_CHECK_HIP(hipIpcCloseMemHandle(base));
  return DQ_OK;
}

int dq_peer_can_access(int32_t device, int32_t peer) {
  if (device == peer) return 1;
  int ok = 0;
  if (hipDeviceCanAccessPeer(&ok, device, peer) != hipSuccess) return 0;
  return ok ? 1 : 0;
}

}  // extern "C"
