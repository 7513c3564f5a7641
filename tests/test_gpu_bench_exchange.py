"""The multi-GPU step of bench.py (encode on the codec stream, RCCL all-gather of the payload on
its own stream and context, double-buffered payloads, then the decode-sum check) rehearsed on one
GPU with a world-size-1 communicator (SKML_BENCH_EXCHANGE=1), so the code the driver's N > 1
runs take is exercised by the GPU suite.  Reference for the exchange:
ml/src/main/scala/org/dma/sketchml/ml/algorithm/GeneralizedLinearModel.scala:145-150.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_exchange_step_world1():
    env = dict(os.environ, SKML_BENCH_EXCHANGE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29541")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--n", str(1 << 22), "--steps", "4",
                          "--warmup", "2", "--no-cpu-baseline", "--no-configs"],
                         capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    ag = line["extras"]["allgather"]
    assert ag["bytes_per_rank"] > 0
    assert ag["decode_sum_max_abs_err_vs_allreduce"] == 0.0
