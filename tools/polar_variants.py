#!/usr/bin/env python3
# Writes the sources of the two k_true_polar-on-the-chain-stream variants of the current engine
# (round-4 experiment for VERDICT r03 item 7): A = the events that mark a
# super-chunk's records final stay on the pooling stream (the round-3 build);
# B = they are recorded after k_true_polar on the chain stream.
import os
import sys
OUT = sys.argv[1] if len(sys.argv) > 1 else '/tmp/tp'
src = open('/root/repo/aperture-robust-multiscale-optical-flow_amd/csrc/farms_engine.hip').read()
src = src.replace('"../../include/farms_hip.h"', '"/root/repo/include/farms_hip.h"')
src = src.replace('#include "farms_libm.h"', '#include "/root/repo/aperture-robust-multiscale-optical-flow_amd/csrc/farms_libm.h"')
old_loop = '''        // (Gx, Gy) -> (RTrue, ThetaTrue): the super-chunk's records are final
        launch_true_polar(h, c, sp, Sg, p0, p1);
        if (int rc = record_pool_done(h, sp, Sg, ev_pool(S))) return rc;
        if (on_super) {
            int rc = (*on_super)(S, p0, p1, ev_pool(S));
            if (rc) return rc;
        }
    }'''
assert src.count(old_loop) == 1
wait_line = '''        if (Sg >= 2) HIPCHK(hipStreamWaitEvent(sc, h->gpool[(Sg - 2) % 3], 0));'''
assert src.count(wait_line) == 1
join = '''    // join: stream F waits for the last chain step and the last pooling launch
    if (n_super > 0) {'''
assert src.count(join) == 1
async_done = '''        HIPCHK(hipEventRecord(w.done, sp));
        w.busy = true;
        return FARMS_OK;
    }'''
assert src.count(async_done) == 1
polar = '''hipLaunchKernelGGL(k_true_polar, dim3(ceil_div(pb1 - pb0, 256)), dim3(256), 0, sc, c, pb0, pb1);'''
def variant(B):
    s = src
    # k_true_polar of super-chunk S - 2 on the chain stream, after its pooling,
    # before the chain of super-chunk S (round 3's arrangement)
    s = s.replace(wait_line, wait_line + '''
        if (S >= 2) {
            const int pb0 = (S - 2) * B * h->pool_chunk, pb1 = (int)std::min<int64_t>((int64_t)(S - 1) * B * h->pool_chunk, n);
            ''' + polar + '''
            ''' + ('HIPCHK(hipEventRecord(w.sync_ev[2 + n_fit_chunks + 2 * (S - 2)], sc));' if B else '') + '''
        }''')
    rec = '''        HIPCHK(hipEventRecord(ev_pool(S), sp));
        HIPCHK(hipEventRecord(h->gpool[Sg % 3], sp));''' if not B else '''        HIPCHK(hipEventRecord(h->gpool[Sg % 3], sp));
        HIPCHK(hipStreamWaitEvent(sc, h->gpool[Sg % 3], 0));  // (the chain stream runs k_true_polar(S) later)'''
    hook = '''        if (on_super) {
            int rc = (*on_super)(S, p0, p1, ev_pool(S));
            if (rc) return rc;
        }''' if not B else ''
    s = s.replace(old_loop, rec + '\n' + hook + '''
    }
    for (int S = std::max(0, n_super - 2); S < n_super; ++S) {  // the last two super-chunks' k_true_polar
        HIPCHK(hipStreamWaitEvent(sc, h->gpool[(sb + S) % 3], 0));
        const int pb0 = S * B * h->pool_chunk, pb1 = (int)std::min<int64_t>((int64_t)(S + 1) * B * h->pool_chunk, n);
        ''' + polar + '''
        ''' + ('HIPCHK(hipEventRecord(ev_pool(S), sc));' if B else '') + '''
    }''' + ('''
    if (on_super)  // (B: the downloads wait for each super-chunk's k_true_polar on the chain stream)
        for (int S = 0; S < n_super; ++S) {
            const int p0 = S * B * h->pool_chunk, p1 = (int)std::min<int64_t>((int64_t)(S + 1) * B * h->pool_chunk, n);
            int rc = (*on_super)(S, p0, p1, ev_pool(S));
            if (rc) return rc;
        }''' if B else ''))
    # the join and the set's done event also wait for the chain stream's tail
    s = s.replace(join, '''    if (n_super > 0) { HIPCHK(hipStreamWaitEvent(s, h->chain_end, 0)); }
''' + join)
    s = s.replace(async_done, '''        HIPCHK(hipStreamWaitEvent(sp, h->chain_end, 0));
''' + async_done)
    return s
open(os.path.join(OUT, 'engA.hip'), 'w').write(variant(False))
open(os.path.join(OUT, 'engB.hip'), 'w').write(variant(True))
# build (container): for v in A B; do hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -shared \
#   -o aperture-robust-multiscale-optical-flow_amd/build/libfarms_hip_polar$v.so $OUT/eng$v.hip; done
