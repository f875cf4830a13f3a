"""The reference's deployment shape: every service in its OWN process (start_all.bat),
here four launcher processes on the CPU with tiny models -- ingest+ui | deid worker |
semantic-indexer | llm-qa -- talking over the multi-process spool bus, a shared SQLite
documents DB and the indexer directory (the llm-qa process follows the indexer's
snapshot + write-ahead log).  A note uploaded to the ingest process becomes INDEXED and
answerable by the llm-qa process without restarting anything."""
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


def _free_offset():
    for off in range(20000, 40000, 97):
        ok = True
        for p in (8000, 8001, 8003, 8005, 8501):
            s = socket.socket()
            try:
                s.bind(("127.0.0.1", p + off))
            except OSError:
                ok = False
            finally:
                s.close()
        if ok:
            return off
    pytest.skip("no free port range")


def _wait(url, deadline):
    while time.time() < deadline:
        try:
            if httpx.get(url, timeout=1.0).status_code == 200:
                return True
        except httpx.HTTPError:
            pass
        time.sleep(0.3)
    return False


def test_services_in_separate_processes(tmp_path):
    off = _free_offset()
    env = dict(os.environ, DOCQA_BUS="spool", DOCQA_SPOOL_DIR=str(tmp_path / "spool"),
               INDEX_DIR=str(tmp_path / "index"), DATABASE_URL=f"sqlite:///{tmp_path}/docs.db",
               DEFAULT_DATA_DIR=str(tmp_path / "nodata"), MAX_NEW_TOKENS="4", PYTHONUNBUFFERED="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    groups = ["ingest,ui", "deid", "indexer", "qa"]
    procs = []
    logs = []
    try:
        for g in groups:
            lf = open(tmp_path / f"{g.replace(',', '_')}.log", "w")
            logs.append(lf)
            procs.append(subprocess.Popen(
                [sys.executable, "-m", "docqa_amd.services.launch", "--tiny", "--device", "cpu",
                 "--services", g, "--port-offset", str(off)], cwd=ROOT, env=env, stdout=lf,
                stderr=subprocess.STDOUT, start_new_session=True))
        deadline = time.time() + 240
        for port in (8000, 8003, 8001):
            assert _wait(f"http://127.0.0.1:{port + off}/health", deadline), \
                (tmp_path / "qa.log").read_text()[-2000:]
        note = ("Compte rendu de consultation. Syndrome de Vide de Qi de la Rate avec fatigue, "
                "digestion lente et selles molles. Traitement: Si Jun Zi Tang pendant quatre semaines. ")
        from docqa_amd.services.multipart import FilePart, encode_multipart

        body, ct = encode_multipart({"file": FilePart("n.txt", "text/plain", note.encode()),
                                     "doc_type": "compte-rendu"})
        r = httpx.post(f"http://127.0.0.1:{8000 + off}/ingest/", content=body,
                       headers={"content-type": ct}, timeout=30)
        doc_id = r.json()["doc_id"]
        status = None
        while time.time() < deadline:
            status = httpx.get(f"http://127.0.0.1:{8000 + off}/documents/{doc_id}", timeout=5).json()["status"]
            if status == "INDEXED":
                break
            time.sleep(0.3)
        assert status == "INDEXED"
        # the question is the indexed chunk itself: its embedding is exact, so it is the
        # nearest neighbour -- proving the llm-qa process sees the new vector
        ans = None
        while time.time() < deadline:
            ans = httpx.post(f"http://127.0.0.1:{8001 + off}/ask/", json={"question": note.strip()},
                             timeout=60).json()
            if ans.get("sources", [None])[0] == f"Dossier Patient {doc_id}":
                break
            time.sleep(0.3)
        assert ans["sources"][0] == f"Dossier Patient {doc_id}", ans
        assert isinstance(ans["answer"], str)
    finally:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        for lf in logs:
            lf.close()


def test_supervisor_restarts_a_dead_service(tmp_path):
    """--supervise runs each group as a child and restarts it after it dies."""
    off = _free_offset()
    env = dict(os.environ, DOCQA_BUS="spool", DOCQA_SPOOL_DIR=str(tmp_path / "spool"),
               INDEX_DIR=str(tmp_path / "index"), DATABASE_URL=f"sqlite:///{tmp_path}/docs.db",
               DEFAULT_DATA_DIR=str(tmp_path / "nodata"), PYTHONUNBUFFERED="1")
    lf = open(tmp_path / "sup.log", "w")
    sup = subprocess.Popen([sys.executable, "-m", "docqa_amd.services.launch", "--tiny", "--device", "cpu",
                            "--port-offset", str(off), "--supervise", "ingest"], cwd=ROOT, env=env,
                           stdout=lf, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        url = f"http://127.0.0.1:{8000 + off}/health"
        assert _wait(url, time.time() + 120)
        # kill the child serving ingest (the supervisor's only child)
        import psutil

        kids = psutil.Process(sup.pid).children()
        assert len(kids) == 1
        kids[0].kill()
        time.sleep(1.0)
        assert _wait(url, time.time() + 120), (tmp_path / "sup.log").read_text()[-2000:]
        assert "restarting" in (tmp_path / "sup.log").read_text()
    finally:
        os.killpg(sup.pid, signal.SIGTERM)
        try:
            sup.wait(timeout=20)
        except subprocess.TimeoutExpired:
            os.killpg(sup.pid, signal.SIGKILL)
        lf.close()
