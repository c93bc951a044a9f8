// threads.h — the host threads a libmando call uses when the caller passes 0: the CPUs this process may
// run on (affinity mask, capped by the cgroup's CPU quota), not std::thread::hardware_concurrency(),
// which on a GPU box is the whole machine (256) while the job's share is 16.
#pragma once
#include <sched.h>

#include <cstdio>
#include <cstdlib>
#include <thread>

namespace mando {
inline int usable_threads() {
    static const int n = [] {
        int c = (int)std::thread::hardware_concurrency();
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) c = CPU_COUNT(&set);
        if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            long long per = 0;
            if (fscanf(f, "%31s %lld", q, &per) == 2 && q[0] != 'm' && per > 0) {
                const long long quota = atoll(q) / per;
                if (quota >= 1 && quota < c) c = (int)quota;
            }
            fclose(f);
        }
        return c > 0 ? c : 1;
    }();
    return n;
}
}  // namespace mando
