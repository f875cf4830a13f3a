"""Container deployment (deploy/Dockerfile, deploy/docker-compose.yml) kept in step with the
launcher and the settings: every service container's command parses with the launcher's
own argument parser, publishes the reference port of the service it runs, and every
environment variable it sets is one the framework reads (reference: docker-compose.yml:1-51,
synthese-comparative/Dockerfile:1-36, start_all.bat:12-35)."""
from __future__ import annotations

import re
from pathlib import Path

import yaml

from docqa_amd.config import Settings
from docqa_amd.services.launch import build_parser

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "docqa_amd"
REF_PORTS = {"ingest": 8000, "qa": 8001, "indexer": 8003, "synthese": 8005, "ui": 8501}
# read outside Settings: by the HIP runtime / the launcher's device-error path
EXTERNAL_ENV = {"HIP_VISIBLE_DEVICES", "DOCQA_EXIT_ON_DEVICE_ERROR"}


def _subst(v: str) -> str:
    """compose's ${VAR:-default} with nothing set: the default."""
    return re.sub(r"\$\{(\w+):-([^}]*)\}", lambda m: m.group(2), str(v))


def _compose() -> dict:
    return yaml.safe_load((ROOT / "deploy" / "docker-compose.yml").read_text())


def _env_names_read() -> set[str]:
    src = "\n".join(p.read_text() for p in PKG.rglob("*.py"))
    return set(re.findall(r"""(?:getenv|environ\.get|env_bool|env_int)\(\s*["'](\w+)["']""", src))


def test_compose_services_match_launcher():
    c = _compose()
    ap = build_parser()
    svcs = {n: s for n, s in c["services"].items() if "command" in s}
    assert set(svcs) == {"doc-ingestor", "deid-service", "semantic-indexer", "llm-qa",
                         "synthese-comparative", "clinical-ui"}
    seen = set()
    for name, s in svcs.items():
        cmd = [_subst(x) for x in s["command"]]
        assert cmd[:3] == ["python", "-m", "docqa_amd.services.launch"], name
        a = ap.parse_args(cmd[3:])
        assert a.host == "0.0.0.0"
        groups = [g for g in a.services.split(",") if g]
        assert len(groups) == 1, name
        seen.add(groups[0])
        if groups[0] in REF_PORTS:
            assert s["ports"] == [f"{REF_PORTS[groups[0]]}:{REF_PORTS[groups[0]]}"], name
        else:
            assert "ports" not in s, name      # the deid worker serves no HTTP
        assert a.gpus % a.tp == 0
        # GPU services pin their devices; CPU-only ones never touch the GPU
        env = s.get("environment", {})
        assert ("HIP_VISIBLE_DEVICES" in env) == (a.device != "cpu"), name
    assert seen == {"ingest", "deid", "indexer", "qa", "synthese", "ui"}


def test_compose_environment_is_read_by_the_framework():
    c = _compose()
    known = _env_names_read() | EXTERNAL_ENV
    for name, s in c["services"].items():
        if "command" not in s:
            continue
        for k in s.get("environment", {}):
            assert k in known, f"{name}: {k} is not read anywhere"
    # the synthese container reaches llm-qa on the port it actually serves
    env = c["services"]["synthese-comparative"]["environment"]
    assert env["LLM_QA_URL"].endswith(f":{REF_PORTS['qa']}")
    assert env["SEMANTIC_INDEXER_URL"].endswith(f":{REF_PORTS['indexer']}")


def test_ui_backend_urls_from_env(monkeypatch):
    assert Settings().ui_ingest_url == "http://127.0.0.1:8000"
    assert Settings().ui_qa_url == "http://127.0.0.1:8001"
    ui_env = _compose()["services"]["clinical-ui"]["environment"]
    for k, v in ui_env.items():
        monkeypatch.setenv(k, str(v))
    st = Settings()
    assert st.ui_ingest_url == "http://doc-ingestor:8000"
    assert st.ui_qa_url == "http://llm-qa:8001"


def test_dockerfile_builds_the_extension_for_gfx950():
    df = (ROOT / "deploy" / "Dockerfile").read_text()
    assert "PYTORCH_ROCM_ARCH=gfx950" in df
    assert "__graft_entry__.py build" in df
    for port in REF_PORTS.values():
        assert str(port) in df.split("EXPOSE", 1)[1].splitlines()[0]
