// pskv_frames.h — the page-locked frame arena behind pskv_host_alloc /
// pskv_host_free (include/pskv.h) and the PSKV_HOST_FRAME call paths.
//
// A frame is a page-locked, device-mapped host buffer handed to the mailbox
// for one message payload (comm/mailbox.cpp:246-257 builds an SArray over each
// received data frame and frees it through the SArray's deleter).  Calls that
// receive frames under PSKV_HOST_FRAME read and write them in place; an Add
// returns once its work is queued, so the arena remembers, per frame, the
// events after which the queued reads have run, and a freed frame goes back to
// its size class only when they have.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace pskv {
namespace frames {

// Allocate a frame of at least `bytes` (0 allowed: one page).  Returns a
// PSKV_* status; *err receives the message of a failure.
int alloc(size_t bytes, void** out, std::string* err);
// Free a frame by the pointer alloc returned.  PSKV_EINVAL for anything else.
int release(void* p, std::string* err);
// Device address of [p, p + bytes) if that range lies inside one live frame,
// else nullptr.
void* device_view(const void* p, size_t bytes);
// Record on `stream` (of the current device `device`) that the frame holding
// p will be read by the work queued so far.  No-op for non-frames.
int note_use(const void* p, int device, hipStream_t stream, std::string* err);
void stats(uint64_t* live, uint64_t* cached, uint64_t* held);
int trim(std::string* err);

}  // namespace frames
}  // namespace pskv
