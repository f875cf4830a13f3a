"""Multi-GPU llm-qa serving, rehearsed on CPU: ``services.launch --gpus 2 --tp 2`` starts two
ranks under torchrun (gloo); TP rank 0 serves HTTP and leads the lockstep continuous-
batching loop, rank 1 mirrors every step with its shard of the generator.  ``/ask/``
answers must be token-exact against the single-process (TP = 1) service: the random init
is TP-invariant, so both hold the same model."""
import json
import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

import httpx
import pytest

ROOT = Path(__file__).resolve().parents[1]
QUESTIONS = ["Quelles plantes pour un vide de Qi de la Rate ?",
             "Patient P00042, 61 ans : insomnie et vertiges depuis 3 semaines, que prescrire ?",
             "Quel est le score de Dang Gui ?"]


def _offset() -> int:
    while True:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if 20000 < p < 50000:
            return p - 8001


def _serve_and_ask(tmp: Path, extra: list[str]) -> list[dict]:
    tmp.mkdir(parents=True, exist_ok=True)
    off = _offset()
    env = dict(os.environ, INDEX_DIR=str(tmp), DATABASE_URL=f"sqlite:///{tmp / 'docs.db'}",
               UPLOAD_DIR=str(tmp / "up"), MAX_NEW_TOKENS="12", MAX_BATCH="8", OMP_NUM_THREADS="2",
               # fp32 weights: TP = 2 sums its row-parallel partials in another order than
               # TP = 1, which in bf16 flips near-tied greedy picks of the random tiny model
               DOCQA_LLM_DTYPE="float32")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    log = open(tmp / "server.log", "w")
    proc = subprocess.Popen([sys.executable, "-m", "docqa_amd.services.launch", "--tiny", "--device", "cpu",
                             "--services", "qa,indexer", "--port-offset", str(off), *extra],
                            cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    url = f"http://127.0.0.1:{8001 + off}"
    try:
        deadline = time.time() + 400
        answers = []
        with httpx.Client(timeout=120) as c:
            while time.time() < deadline:
                assert proc.poll() is None, (tmp / "server.log").read_text()[-3000:]
                try:
                    r = c.post(url + "/ask/", json={"question": QUESTIONS[0]})
                    if r.status_code == 200:
                        break
                except httpx.HTTPError:
                    pass
                time.sleep(1.0)
            for q in QUESTIONS:
                r = c.post(url + "/ask/", json={"question": q})
                assert r.status_code == 200, r.text
                answers.append(r.json())
        return answers
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait()
        log.close()


@pytest.mark.slow
def test_ask_tp2_service_matches_tp1(tmp_path):
    one = _serve_and_ask(tmp_path / "tp1", [])
    two = _serve_and_ask(tmp_path / "tp2", ["--gpus", "2", "--tp", "2"])
    assert [a["answer"] for a in two] == [a["answer"] for a in one], json.dumps([one, two])[:2000]
    assert [a["sources"] for a in two] == [a["sources"] for a in one]
    assert all(a["answer"] for a in one)
