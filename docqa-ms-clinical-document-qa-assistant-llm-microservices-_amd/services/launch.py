"""Run the DocQA stack: every service on the reference's port, one process per GPU.

    python -m docqa_amd.services.launch                 # full stack on cuda:0
    python -m docqa_amd.services.launch --tiny --device cpu   # CPU demo with tiny models

Ports (start_all.bat:18,31; synthese Dockerfile:27,36; clinical-ui Streamlit default):
doc-ingestor 8000, llm-qa 8001, semantic-indexer 8003, synthese-comparative 8005, UI 8501.
"""
from __future__ import annotations

import argparse
import logging
import threading

import uvicorn

from .stack import DocQAStack, StackOptions


def serve(app, port: int, host: str) -> threading.Thread:
    cfg = uvicorn.Config(app, host=host, port=port, log_level="warning")
    server = uvicorn.Server(cfg)
    t = threading.Thread(target=server.run, name=f"uvicorn-{port}", daemon=True)
    t.start()
    return t


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--tiny", action="store_true", help="tiny random models (CPU demo / CI)")
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--embed", default="minilm-l6")
    ap.add_argument("--real-synthese", action="store_true")
    a = ap.parse_args()
    logging.basicConfig(level=logging.INFO)
    opts = StackOptions(llm="tiny" if a.tiny else a.llm, embed="tiny-bert" if a.tiny else a.embed,
                        ner="tiny-bert" if a.tiny else "clinical-bert", device=a.device,
                        use_graphs=a.device != "cpu", max_context=2048 if a.tiny else 4096,
                        real_synthese=a.real_synthese)
    stack = DocQAStack(opts)
    threads = [serve(stack.ingest_app, 8000, a.host), serve(stack.qa_app, 8001, a.host),
               serve(stack.indexer_app, 8003, a.host), serve(stack.synthese_app, 8005, a.host),
               serve(stack.ui_app, 8501, a.host)]
    print("DocQA stack up: ingest :8000, llm-qa :8001, indexer :8003, synthese :8005, ui :8501", flush=True)
    try:
        for t in threads:
            t.join()
    except KeyboardInterrupt:
        stack.close()


if __name__ == "__main__":
    main()
