// tests/test_user_stack_registry.py: hip_backend.h's process-wide maximum depth of the BVHs a program
// has taken refs of (hip_index_bvh::ref -> note_ref_depth), which decides whether a user-kernel launch
// gives its threads the short LDS stack (hip_kernels.h VRH_USER_LDS_STACK): starts at 0, only grows,
// and keeps the maximum when threads note depths at once.  Host code only (no GPU, no libvrh calls).
#include <visionaray_hip/hip_backend.h>
#include <cstdio>
#include <thread>
#include <vector>
int main()
{
    using namespace visionaray::hip_detail;
    if (user_ref_depth().load() != 0u) return 1;
    note_ref_depth(20); note_ref_depth(12);
    if (user_ref_depth().load() != 20u) return 2;
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < 8; ++t) ts.emplace_back([t] { for (unsigned d = 0; d < 10000; ++d) note_ref_depth((d * 7 + t) % 31); });
    for (auto& th : ts) th.join();
    if (user_ref_depth().load() != 30u) return 3;
    printf("ok %u\n", user_ref_depth().load());
    return 0;
}
