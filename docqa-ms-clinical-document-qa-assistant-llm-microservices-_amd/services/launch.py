"""Run the DocQA stack: every service on the reference's port, one process per GPU, or
one process per service like the reference's start_all.bat.

    python -m docqa_amd.services.launch                 # full stack on cuda:0
    python -m docqa_amd.services.launch --tiny --device cpu   # CPU demo with tiny models
    # microservices, one process each (shared spool bus, SQLite file, index directory):
    export DOCQA_BUS=spool DOCQA_SPOOL_DIR=/srv/docqa/spool INDEX_DIR=/srv/docqa/index \
           DATABASE_URL=sqlite:////srv/docqa/docs.db
    python -m docqa_amd.services.launch --services ingest
    python -m docqa_amd.services.launch --services deid --device cuda:1
    python -m docqa_amd.services.launch --services indexer --device cuda:2
    python -m docqa_amd.services.launch --services qa,ui --device cuda:3
    # multi-GPU llm-qa (one process per GPU under torchrun, spawned by this launcher):
    python -m docqa_amd.services.launch --gpus 8 --tp 8 --llm llama3-70b   # one TP=8 group
    python -m docqa_amd.services.launch --gpus 8 --tp 2                     # 4 DP replicas x TP=2

Multi-GPU layout (``--gpus N --tp T``): N / T data-parallel replicas of a T-way
tensor-parallel generator.  Within a TP group, TP rank 0 serves HTTP and leads a lockstep
continuous-batching loop (engine/scheduler.py Lockstep: arrivals + the admission decision
broadcast before every step over a gloo group) that the other ranks mirror, each running
its shard of every TP forward.  Replica 0's leader hosts every requested service on the
reference ports and balances ``/ask/`` and ``/api/llm/summarize`` over the replicas;
replica d's leader serves llm-qa on port 8001 + 100 d over the indexer's shared snapshot
(index/follower.py).

Ports (start_all.bat:18,31; synthese Dockerfile:27,36; clinical-ui Streamlit default):
doc-ingestor 8000, llm-qa 8001, semantic-indexer 8003, synthese-comparative 8005, UI 8501.
"""
from __future__ import annotations

import argparse
import logging
import threading

import uvicorn

from ..config import Settings
from .stack import DocQAStack, StackOptions


def serve(app, port: int, host: str) -> threading.Thread:
    # keep-alive longer than a client's idle gap between bursts: at uvicorn's 5 s default the
    # server closes pooled connections just as a Poisson client reuses them (ReadError)
    cfg = uvicorn.Config(app, host=host, port=port, log_level="warning", timeout_keep_alive=75,
                         backlog=4096)
    server = uvicorn.Server(cfg)
    t = threading.Thread(target=server.run, name=f"uvicorn-{port}", daemon=True)
    t.start()
    return t


def supervise(groups: list[str], argv: list[str], max_restarts: int = 10, backoff_s: float = 1.0) -> None:
    """Run each service group as a child process and restart it when it dies (SURVEY.md
    §5.3: the reference only retries its AMQP connection every 5 s; a process whose GPU
    context is poisoned -- a sticky HIP error -- can only be recovered by a restart).
    Children get DOCQA_EXIT_ON_DEVICE_ERROR=1 so a device fault ends them promptly."""
    import os
    import subprocess
    import sys
    import time

    env = dict(os.environ, DOCQA_EXIT_ON_DEVICE_ERROR="1")
    procs: dict[str, subprocess.Popen] = {}
    restarts = {g: 0 for g in groups}
    next_start = {g: 0.0 for g in groups}

    def spawn(g: str) -> subprocess.Popen:
        print(f"[supervisor] starting {g}", flush=True)
        return subprocess.Popen([sys.executable, "-m", "docqa_amd.services.launch", *argv, "--services", g], env=env)

    for g in groups:
        procs[g] = spawn(g)
    try:
        while procs:
            time.sleep(0.5)
            for g, p in list(procs.items()):
                rc = p.poll()
                if rc is None:
                    continue
                if restarts[g] >= max_restarts:
                    print(f"[supervisor] {g} exited {rc}; restart budget spent", flush=True)
                    del procs[g]
                    continue
                now = time.monotonic()
                if next_start[g] == 0.0:
                    next_start[g] = now + backoff_s * (2 ** restarts[g])
                    print(f"[supervisor] {g} exited {rc}; restarting", flush=True)
                if now >= next_start[g]:
                    restarts[g] += 1
                    next_start[g] = 0.0
                    procs[g] = spawn(g)
    except KeyboardInterrupt:
        for p in procs.values():
            p.terminate()


def _free_port() -> int:
    import socket

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def spawn_workers(gpus: int, argv: list[str]) -> int:
    """Start this launcher once per GPU under torchrun (a child process: nothing here has
    touched the GPU) and return its exit code."""
    import subprocess
    import sys

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m",
           "docqa_amd.services.launch", *argv]
    p = subprocess.Popen(cmd)
    try:
        return p.wait()
    except KeyboardInterrupt:       # torchrun got the same SIGINT and shuts the ranks down
        try:
            return p.wait(timeout=120)
        except subprocess.TimeoutExpired:
            p.kill()
            return p.wait()


def run_parallel(a, opts: "StackOptions") -> None:
    """One rank of ``--gpus N --tp T`` (under torchrun)."""
    import os
    import time

    import torch

    from ..engine.llm_engine import LLMEngine
    from ..engine.scheduler import ContinuousEngine, Lockstep
    from ..config import Settings
    from ..models import checkpoint as ck
    from ..parallel import comm

    cuda = a.device != "cpu"
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if cuda:
        torch.cuda.set_device(local)
        opts.device = f"cuda:{local}"
    ps = comm.init_distributed(tp_size=a.tp, backend=None if cuda else "gloo")
    torch.manual_seed(1234)    # identical sampling streams on every rank of a TP group
    ls = None
    if ps.tp_size > 1:
        ls = Lockstep(ps.tp_cpu_group, src=ps.dp_rank * ps.tp_size, leader=ps.tp_rank == 0)
    st = Settings()
    o = a.port_offset
    if ps.tp_rank != 0:
        # follower: only this rank's shard of the generator, mirroring the leader's steps.
        # Shutdown is the leader's "stop" message (a Ctrl-C reaches every rank at once;
        # a follower that died first would leave the leader's last broadcast hanging).
        import signal

        signal.signal(signal.SIGINT, signal.SIG_IGN)
        ck.use_checkpoint_tokenizers(opts.llm, opts.embed)
        model = ck.resolve_llama(opts.llm, device=opts.device)
        ctx = min(opts.max_context or st.max_context, model.cfg.max_position)
        eng = LLMEngine(model, max_batch=opts.max_batch, max_context=ctx, use_graphs=opts.use_graphs,
                        kv_mem_fraction=opts.kv_mem_fraction)
        ce = ContinuousEngine(eng, max_running=st.max_batch, lockstep=ls)
        if os.environ.get("DOCQA_WARM_BUCKETS", "1") == "1":
            ce.warmup()        # the leader captures the same buckets in the same order (qa.py)
        print(f"[rank {ps.rank}] TP follower of group {ps.dp_rank} ready", flush=True)
        ce.follow()
        comm.destroy()
        return
    opts.qa_lockstep = ls
    apps_ports = []
    if ps.dp_rank == 0:
        opts.qa_replicas = tuple(f"http://{a.host}:{8001 + o + 100 * d}" for d in range(1, ps.dp_size))
        stack = DocQAStack(opts)
        apps_ports = [(stack.ingest_app, 8000), (stack.qa_app, 8001), (stack.indexer_app, 8003),
                      (stack.synthese_app, 8005), (stack.ui_app, 8501)]
    else:
        opts.services = ("qa",)
        stack = DocQAStack(opts)
        apps_ports = [(stack.qa_app, 8001 + 100 * ps.dp_rank)]
    threads = [serve(app, port + o, a.host) for app, port in apps_ports if app is not None]
    print(f"DocQA rank {ps.rank} (replica {ps.dp_rank}, TP {ps.tp_size}) up: "
          + ", ".join(f":{port + o}" for app, port in apps_ports if app is not None), flush=True)
    try:
        while any(t.is_alive() for t in threads):
            time.sleep(1.0)
    except KeyboardInterrupt:
        pass
    stack.close()
    comm.destroy()


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--tiny", action="store_true", help="tiny random models (CPU demo / CI)")
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--embed", default="minilm-l6")
    ap.add_argument("--real-synthese", action="store_true")
    ap.add_argument("--services", default="", help="comma list of ingest,deid,indexer,qa,synthese,ui (default all)")
    ap.add_argument("--port-offset", type=int, default=0, help="added to every reference port (tests)")
    ap.add_argument("--supervise", default="", help='service groups, one child process each, restarted '
                    'when they die: e.g. "ingest,ui;deid;indexer;qa"')
    ap.add_argument("--gpus", type=int, default=1, help="GPUs (one process each, torchrun)")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel size of the generator (divides --gpus)")
    ap.add_argument("--preload-notes", type=int, default=0,
                    help="index this many synthetic clinical notes at start (serving benchmarks, demos)")
    ap.add_argument("--kv-mem-fraction", type=float, default=0.8, help="KV pool share of free HBM")
    ap.add_argument("--deid-ner", choices=("auto", "on", "off"), default=None,
                    help="NER token classifier in the deid worker (default: env DEID_NER, auto = when "
                         "NER_CHECKPOINT names a checkpoint)")
    ap.add_argument("--ner-checkpoint", default=None, help="BERT token-classification checkpoint (NER_CHECKPOINT)")
    return ap


def main() -> None:
    a = build_parser().parse_args()
    import os
    import sys

    # The HTTP front end (uvicorn thread), the QA prep thread and the engine's scheduler
    # thread share one GIL; at CPython's 5 ms switch interval each request's few GIL hand-
    # offs queue behind the scheduler's per-step Python, throttling admissions under load.
    # DOCQA_GIL_SWITCH_MS (default 0.5) shortens the hand-off wait.
    sys.setswitchinterval(float(os.environ.get("DOCQA_GIL_SWITCH_MS", "0.5")) / 1e3)
    under_torchrun = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if a.gpus > 1 and not under_torchrun:
        if a.gpus % a.tp:
            raise SystemExit("--tp must divide --gpus")
        sys.exit(spawn_workers(a.gpus, sys.argv[1:]))
    if a.supervise:
        import sys

        argv = [x for x in sys.argv[1:]]
        i = argv.index("--supervise")
        del argv[i:i + 2]
        supervise([g for g in a.supervise.split(";") if g], argv)
        return
    logging.basicConfig(level=logging.INFO)
    if a.deid_ner is not None:
        os.environ["DEID_NER"] = {"on": "1", "off": "0"}.get(a.deid_ner, "auto")
    if a.ner_checkpoint:
        os.environ["NER_CHECKPOINT"] = a.ner_checkpoint
    opts = StackOptions(llm="tiny" if a.tiny else a.llm, embed="tiny-bert" if a.tiny else a.embed,
                        ner="tiny-bert" if a.tiny else "clinical-bert", device=a.device,
                        use_graphs=a.device != "cpu", max_context=2048 if a.tiny else None,
                        real_synthese=a.real_synthese,
                        services=tuple(x for x in a.services.split(",") if x),
                        max_batch=Settings().max_batch, preload_notes=a.preload_notes,
                        kv_mem_fraction=a.kv_mem_fraction)
    if under_torchrun:
        run_parallel(a, opts)
        return
    stack = DocQAStack(opts)
    o = a.port_offset
    apps = [("ingest", stack.ingest_app, 8000), ("llm-qa", stack.qa_app, 8001),
            ("indexer", stack.indexer_app, 8003), ("synthese", stack.synthese_app, 8005),
            ("ui", stack.ui_app, 8501)]
    threads = [serve(app, port + o, a.host) for _, app, port in apps if app is not None]
    up = ", ".join(f"{n} :{port + o}" for n, app, port in apps if app is not None)
    extra = " (+ deid worker)" if stack.deid is not None else ""
    print(f"DocQA up: {up or 'no HTTP service'}{extra}", flush=True)
    if not threads:   # worker-only process (deid): keep it alive
        import time
        while True:
            time.sleep(3600)
    try:
        for t in threads:
            t.join()
    except KeyboardInterrupt:
        stack.close()


if __name__ == "__main__":
    main()
