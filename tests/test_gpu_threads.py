"""GPU: several event-loop threads drive the drop-in at once (SURVEY.md
sec. 8(b): "callable from multiple loop threads at once ... per-thread or
per-device contexts and HIP streams, with no global device lock").  Each
thread owns its connections and feeds them with hvws_wsp_feed_many, its own
pipelined feeder, or per-read hvws_wsp_feed while the others do the same; every connection must
end exactly as the reference's sequential FeedRecvData would leave it.
ctypes releases the GIL around foreign calls, so the library calls overlap."""
from __future__ import annotations

import random
import threading

import pytest

import streams as S
from test_gpu_feed_many import Conn, _check, _loop

import libhv_amd

pytestmark = pytest.mark.gpu


def _worker(seed, conns_out, errors, per_read, feeder=False):
    try:
        rng = random.Random(seed)
        conns = []
        for _ in range(rng.randint(4, 24)):
            data = S.rand_stream(rng, rng.randint(1, 12), max_len=rng.choice([60, 600, 20000]))
            conns.append(Conn(data, S.rand_chunks(rng, len(data), rng.choice(["rand", "small", "one"]))))
        if per_read:
            L = libhv_amd.lib()
            import ctypes
            for c in conns:
                for k in list(c.chunks):
                    c.rets.append(L.hvws_wsp_feed(c.h, ctypes.addressof(c.buf) + c.at, k))
                    c.at += k
                c.chunks = []
        else:
            _loop(rng, conns, feeder=feeder)   # a feeder of its own per loop thread
        conns_out.extend(conns)
        libhv_amd.lib().hvws_thread_release()   # loop-thread exit
    except Exception as e:  # noqa: BLE001 -- reported by the main thread
        errors.append(e)


@pytest.mark.parametrize("feeder", [False, True], ids=["many", "feeders"])
@pytest.mark.parametrize("nthreads", [2, 6])
def test_concurrent_loop_threads(nthreads, feeder):
    outs = [[] for _ in range(nthreads)]
    errors = []
    ts = [threading.Thread(target=_worker, args=(100 + t, outs[t], errors, t % 3 == 2, feeder))
          for t in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errors, errors
    for conns in outs:
        _check(conns)
