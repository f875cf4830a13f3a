"""clinical-ui: a dependency-free web page (FastAPI-served HTML + fetch) replacing the
reference's Streamlit app (clinical-ui/app.py:1-118): sidebar health probes
(``GET {url}/health``, 2 s timeout), document upload to ``POST /ingest/`` with
``doc_type="compte-rendu"`` and readiness polling of ``GET /documents/{id}`` (instead of
a fixed 5 s sleep), and a chat box posting ``{"question"}`` to ``/ask/`` that renders the
answer and its sources.  The page proxies to the services through the UI server so the
browser never needs CORS."""
from __future__ import annotations

import httpx
from fastapi import FastAPI, Request
from fastapi.responses import HTMLResponse, JSONResponse, Response

PAGE = """<!doctype html><html lang="fr"><head><meta charset="utf-8">
<title>Assistant Clinique (MI355X)</title>
<style>body{font-family:sans-serif;display:flex;margin:0}#side{width:280px;background:#f4f6f8;padding:16px;height:100vh}
#main{flex:1;padding:16px}.msg{margin:8px 0;padding:8px;border-radius:6px}.u{background:#e3f2fd}.a{background:#f1f8e9}
.src{font-size:12px;color:#555}.ok{color:green}.ko{color:red}</style></head><body>
<div id="side"><h3>Services</h3><div id="health"></div><h3>Documents</h3>
<input type="file" id="f" accept=".pdf,.txt,.docx"><button onclick="up()">Traiter et Ingérer</button><div id="st"></div></div>
<div id="main"><h2>Assistant de questions cliniques</h2><div id="chat"></div>
<input id="q" style="width:70%" placeholder="Votre question..."><button onclick="ask()">Envoyer</button></div>
<script>
async function health(){const r=await fetch('/ui/health');const j=await r.json();
document.getElementById('health').innerHTML=Object.entries(j).map(([k,v])=>`<div class="${v?'ok':'ko'}">${k}: ${v?'en ligne':'hors ligne'}</div>`).join('')}
async function up(){const f=document.getElementById('f').files[0];if(!f)return;const fd=new FormData();fd.append('file',f);fd.append('doc_type','compte-rendu');
const st=document.getElementById('st');st.textContent='Envoi...';const r=await fetch('/ui/ingest',{method:'POST',body:fd});const j=await r.json();
if(!j.doc_id){st.textContent='Erreur: '+(j.error||JSON.stringify(j));return}
for(let i=0;i<120;i++){const d=await (await fetch('/ui/documents/'+j.doc_id)).json();st.textContent='Statut: '+d.status;if(d.status==='INDEXED'||String(d.status).startsWith('ERROR'))break;await new Promise(r=>setTimeout(r,500))}}
async function ask(){const q=document.getElementById('q').value;if(!q)return;const c=document.getElementById('chat');
c.innerHTML+=`<div class="msg u">${q}</div>`;const r=await fetch('/ui/ask',{method:'POST',headers:{'Content-Type':'application/json'},body:JSON.stringify({question:q})});
const j=await r.json();c.innerHTML+=`<div class="msg a">${(j.answer||j.detail||'').replace(/</g,'&lt;')}<div class="src">Sources: ${(j.sources||[]).join(', ')}</div></div>`}
health();setInterval(health,10000);
</script></body></html>"""


def create_app(ingest_url: str = "http://127.0.0.1:8000", qa_url: str = "http://127.0.0.1:8001") -> FastAPI:
    app = FastAPI(title="Clinical UI")

    @app.get("/", response_class=HTMLResponse)
    def index():
        return PAGE

    @app.get("/ui/health")
    async def health():
        out = {}
        async with httpx.AsyncClient(timeout=2.0) as c:
            for name, url in (("doc-ingestor", ingest_url), ("llm-qa", qa_url)):
                try:
                    out[name] = (await c.get(f"{url}/health")).status_code == 200
                except Exception:  # noqa: BLE001
                    out[name] = False
        return out

    @app.post("/ui/ingest")
    async def ingest(request: Request):
        body = await request.body()
        async with httpx.AsyncClient(timeout=120.0) as c:
            r = await c.post(f"{ingest_url}/ingest/", content=body,
                             headers={"content-type": request.headers.get("content-type", "")})
        return Response(content=r.content, status_code=r.status_code, media_type="application/json")

    @app.get("/ui/documents/{doc_id}")
    async def doc(doc_id: int):
        async with httpx.AsyncClient(timeout=5.0) as c:
            r = await c.get(f"{ingest_url}/documents/{doc_id}")
        return JSONResponse(status_code=r.status_code, content=r.json())

    @app.post("/ui/ask")
    async def ask(request: Request):
        async with httpx.AsyncClient(timeout=600.0) as c:
            r = await c.post(f"{qa_url}/ask/", json=await request.json())
        return JSONResponse(status_code=r.status_code, content=r.json())

    return app
