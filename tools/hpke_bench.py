# Batched helper HPKE open rate vs host threads (tools/hpke_bench.py 1,8,16 [scalar]: 'scalar' = the
# scalar X25519 ladder for every report, prio3gpu_test_hpke_set_ifma(0))
import sys, time, os
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
import numpy as np
from janus_amd import codec as C, hpke as H
from test_hpke import _request
rng=np.random.default_rng(1); n=4096
task_id=bytes(32); tk=H.generate_hpke_config_and_private_key(1)
nonces=rng.integers(0,256,(n,16),dtype=np.uint8); public=rng.integers(0,256,(n,32),dtype=np.uint8)
payloads=[bytes(48) for _ in range(n)]
if len(sys.argv) > 2 and sys.argv[2] == 'scalar':
    from janus_amd._lib import lib
    lib().prio3gpu_test_hpke_set_ifma(0)
req=C.decode_agg_init_req(_request(task_id,nonces,[0]*n,public,payloads,[tk]*n))
for th in [int(x) for x in sys.argv[1].split(",")]:
    H.open_report_shares(task_id,req,[tk],[],None,th)
    t=time.perf_counter(); r=0
    while time.perf_counter()-t<1.5:
        _,_,st=H.open_report_shares(task_id,req,[tk],[],None,th); r+=1
    dt=time.perf_counter()-t; assert (st==0).all()
    print(th, f"{r*n/dt:.0f} opens/s  {dt/(r*n)*th*1e6:.1f} us/open/thread")
