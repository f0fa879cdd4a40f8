"""The torchrun serving entry point with data-parallel replicas (`llmss_amd/serving/server.py _serve_replicas`): a
dp=2 x tp=1 world on gloo / CPU. Global rank 0 hosts the broker (asyncio MiniRedisServer) and the coroutine gRPC
front-end (AioBrokerServicer); both replica leaders pull from the broker through their consumers. Concurrent gRPC
requests get the offline engine's greedy continuations."""
import concurrent.futures as cf
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import grpc

from helpers import save_hf_model


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_torchrun_dp2_server_serves_through_the_broker(tmp_path):
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.serving.grpc_api import GenerateRequest, Stub
    from llmss_amd.utils.tokenizer import encode, load_tokenizer

    d = str(tmp_path / "gpt2")
    save_hf_model("gpt2", d, vocab=101, with_tokenizer=True)
    gport, bport, mport = _free_port(), _free_port(), _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={mport}", "-m", "llmss_amd.serving.server", "--model", d, "--grpc_host", "127.0.0.1",
           "--grpc_port", str(gport), "--broker_port", str(bport), "--dp", "2", "--max_num_seqs", "4",
           "--block_size", "4", "--no_graphs", "--dtype", "fp32"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               PYTHONPATH=os.pathsep.join([os.getcwd(), os.environ.get("PYTHONPATH", "")]))
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env,
                         start_new_session=True)
    lines, ready = [], threading.Event()

    def pump():
        for ln in p.stdout:
            lines.append(ln)
            if "gRPC Generate on" in ln:
                ready.set()

    threading.Thread(target=pump, daemon=True).start()
    try:
        assert ready.wait(180), "".join(lines[-40:])
        tok = load_tokenizer(d, 101)
        prompts = [f"tiny prompt {i}" for i in range(8)]
        ref = LLMEngine(build_model(d, None, "fp32", "cpu"), max_num_seqs=4, block_size=4, num_blocks=256,
                        eos_token_id=None)
        want = ref.generate([encode(tok, q) for q in prompts], SamplingParams(max_new_tokens=5, is_greedy=True,
                                                                               ignore_eos=True))
        stub = Stub(grpc.insecure_channel(f"127.0.0.1:{gport}"))
        with cf.ThreadPoolExecutor(8) as ex:
            outs = list(ex.map(lambda q: stub.Generate(GenerateRequest(prompt=q, max_new_tokens=5, is_greedy=True,
                                                                       ignore_eos=True), timeout=120), prompts))
        assert [list(o.token_ids) for o in outs] == want
        assert all(o.prompt == q for o, q in zip(outs, prompts))
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        t0 = time.time()
        while p.poll() is None and time.time() - t0 < 20:
            time.sleep(0.2)
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(10)
