// in_tree_frames.cpp — compiles include/ps/host_frames.hpp in its
// PSKV_IN_REFERENCE_TREE form against the reference's own boundary types
// (base/third_party/sarray.h, base/message.hpp), as INTEGRATION.md §2 tells a
// maintainer to include it.  Built and linked by tests/test_in_tree.py (CPU;
// never run there: pskv_host_alloc needs a GPU).
#define PSKV_IN_REFERENCE_TREE 1

#include "base/message.hpp"
#include "ps/host_frames.hpp"

#include <cstdio>
#include <utility>

int main() {
  using csci5570::third_party::SArray;
  // a Get reply frame, as HipStorage::SubGet allocates it, reinterpreted as the
  // reply's SArray<char> (the explicit converting constructor, sarray.h:67-68)
  SArray<float> vals = csci5570::FrameArray<float>(16);
  SArray<char> bytes(vals);
  // a received data frame (Mailbox::Recv, comm/mailbox.cpp:246-257), carried in
  // a reference Message as its key payload
  const uint32_t keys[4] = {13, 14, 15, 16};
  SArray<char> frame = csci5570::RecvIntoFrame(keys, sizeof(keys));
  csci5570::Message m;
  m.meta.flag = csci5570::Flag::kGet;
  m.AddData(SArray<csci5570::Key>(frame));
  std::printf("%zu %zu %zu\n", (size_t)bytes.size(), (size_t)m.data.size(),
              (size_t)SArray<csci5570::Key>(m.data[0]).size());
  return 0;
}
