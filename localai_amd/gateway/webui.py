"""Built-in web UI (`core/http/routes/ui.go:87-432`, `core/http/views/*.html` -- behaviour, not
assets): home page with the installed models (loaded state, backend monitor, unload), model
gallery browser with search, install/delete and job progress, streaming chat (system prompt,
sampling knobs, image attachments for vision models, code blocks), text-to-speech (voice /
backend), text-to-image (size, steps, seed, negative prompt, result gallery), sound generation
and the push-to-talk loop; the P2P page lives with the p2p routes (gateway/p2p.py).

Self-contained HTML + vanilla JS served by the gateway (no build step, no CDN: the server may
run air-gapped).  Every page talks to the public REST API (/v1/chat/completions with SSE,
/models/apply, /models/jobs/:uuid, /tts, /v1/images/generations), so the UI exercises exactly
the endpoints clients use.  `/` keeps the JSON welcome document for API clients (Accept:
application/json), like the reference's content negotiation.  Disabled by --disable-webui.
"""
from __future__ import annotations

import html
import time
import urllib.parse

from fastapi import APIRouter, Request
from fastapi.responses import HTMLResponse, JSONResponse

from .. import __version__

_CSS = """
body{font-family:system-ui,sans-serif;margin:0;background:#0f1115;color:#e6e6e6}
header{display:flex;gap:1.2em;align-items:center;padding:.7em 1.2em;background:#171a21;border-bottom:1px solid #2a2f3a}
header b{color:#ff7a45}header a{color:#cfd6e4;text-decoration:none}header a:hover{color:#fff}
main{max-width:980px;margin:1.2em auto;padding:0 1em}
table{border-collapse:collapse;width:100%}td,th{border-bottom:1px solid #2a2f3a;padding:.45em;text-align:left}
button,select,input,textarea{background:#1f2430;color:#e6e6e6;border:1px solid #39404f;border-radius:6px;padding:.45em .7em}
button{cursor:pointer}button:hover{background:#2b3242}
#log{white-space:pre-wrap;background:#151821;border:1px solid #2a2f3a;border-radius:8px;padding:1em;min-height:260px}
.u{color:#8ab4ff}.a{color:#e6e6e6}.muted{color:#8a93a5;font-size:.9em}
.row{display:flex;gap:.6em;margin:.8em 0}.row>*{flex:1}.row>button,.row>select{flex:0 0 auto}
pre.code{background:#0b0d12;border:1px solid #2a2f3a;border-radius:6px;padding:.6em;overflow-x:auto}
.card{border:1px solid #2a2f3a;border-radius:8px;padding:.6em 1em;margin:.6em 0}.tag{background:#1f2430;border-radius:4px;padding:0 .4em;margin-right:.3em;font-size:.85em}
.progress{background:#1f2430;border-radius:4px;height:10px;width:60%;display:inline-block}.progress .bar{background:#ff7a45;height:10px;border-radius:4px}
.grid{display:grid;grid-template-columns:repeat(auto-fill,minmax(220px,1fr));gap:.8em}.grid img{width:100%;border-radius:6px}
label{color:#8a93a5;font-size:.9em;align-self:center}
"""

_NAV = ('<header><b>LocalAI · MI355X</b><a href="/">Home</a><a href="/browse">Models</a>'
        '<a href="/chat/">Chat</a><a href="/tts/">TTS</a><a href="/text2image/">Text→Image</a>'
        '<a href="/sound/">Sound</a><a href="/talk/">Talk</a><a href="/p2p">P2P</a>'
        '<a href="/swagger">API</a></header>')


def _page(title: str, body: str, script: str = "") -> HTMLResponse:
    return HTMLResponse(f"<!doctype html><html><head><meta charset='utf-8'><title>{html.escape(title)}</title>"
                        f"<style>{_CSS}</style></head><body>{_NAV}<main>{body}</main>"
                        f"<script>{script}</script></body></html>")


def _model_select(models, selected: str, id_: str = "model") -> str:
    opts = "".join(f"<option{' selected' if m == selected else ''}>{html.escape(m)}</option>" for m in models)
    return f"<select id='{id_}'>{opts}</select>"


_AUTH_JS = """
const KEY = localStorage.getItem('localai_key') || '';
function hdrs(){const h={'Content-Type':'application/json'}; if(KEY) h['Authorization']='Bearer '+KEY; return h;}
"""

_CHAT_JS = _AUTH_JS + """
const log = document.getElementById('log'), inp = document.getElementById('msg');
let history = [], image = null;
function add(cls, text){const d=document.createElement('div'); d.className=cls; d.textContent=text; log.appendChild(d); return d;}
// fenced code blocks of a reply as <pre> elements; everything stays text (no HTML injection)
function render(el, text){
  el.textContent = ''; const parts = text.split('```');
  parts.forEach((p, i) => { const n = document.createElement(i % 2 ? 'pre' : 'span');
    n.textContent = i % 2 ? p.replace(/^[a-zA-Z0-9_+-]*\n/, '') : p; if(i % 2) n.className = 'code'; el.appendChild(n); });
}
function num(id){ const v = document.getElementById(id).value; return v === '' ? undefined : parseFloat(v); }
function clearChat(){ history = []; log.textContent = ''; image = null; document.getElementById('img').value = ''; }
document.getElementById('img').addEventListener('change', e => {
  const f = e.target.files[0]; if(!f) { image = null; return; }
  const r = new FileReader(); r.onload = () => { image = r.result; }; r.readAsDataURL(f);
});
async function send(){
  const text = inp.value.trim(); if(!text) return; inp.value='';
  const sys = document.getElementById('sys').value.trim();
  const content = image ? [{type:'text', text}, {type:'image_url', image_url:{url:image}}] : text;
  history.push({role:'user', content}); add('u', '> ' + text + (image ? '  [image]' : ''));
  image = null; document.getElementById('img').value = '';
  const msgs = sys ? [{role:'system', content:sys}].concat(history) : history;
  const out = add('a', ''); const t0 = performance.now(); let first = 0, n = 0;
  const res = await fetch('/v1/chat/completions', {method:'POST', headers:hdrs(), body: JSON.stringify({
    model: document.getElementById('model').value, messages: msgs, stream: true,
    temperature: num('temp'), top_p: num('topp'), max_tokens: num('maxt') && Math.round(num('maxt'))})});
  if(!res.ok){out.textContent = 'error: ' + res.status + ' ' + await res.text(); return;}
  const rd = res.body.getReader(), dec = new TextDecoder(); let buf = '', full = '';
  for(;;){
    const {value, done} = await rd.read(); if(done) break;
    buf += dec.decode(value, {stream:true});
    let i; while((i = buf.indexOf('\\n')) >= 0){
      const line = buf.slice(0, i).trim(); buf = buf.slice(i + 1);
      if(!line.startsWith('data:')) continue; const data = line.slice(5).trim();
      if(data === '[DONE]') continue;
      try{const j = JSON.parse(data); const d = (j.choices && j.choices[0].delta) || {};
          if(d.content){ if(!first) first = performance.now(); n++; full += d.content; render(out, full); }}catch(e){}
    }
  }
  history.push({role:'assistant', content: full});
  const s = (performance.now() - t0) / 1000;
  document.getElementById('stats').textContent =
    `TTFT ${first ? ((first - t0)).toFixed(0) : '-'} ms · ${n} chunks · ${(n / Math.max(s, 1e-3)).toFixed(1)} chunks/s`;
}
inp.addEventListener('keydown', e => { if(e.key === 'Enter' && !e.shiftKey){ e.preventDefault(); send(); } });
"""

_BROWSE_JS = _AUTH_JS + """
// The gallery actions talk to the reference's htmx routes (core/http/routes/ui.go:169-300):
// POST /browse/search/models -> card list fragment, POST /browse/install|delete/model/:id ->
// progress fragment, GET /browse/job/progress/:uid every 600 ms until the response carries
// HX-Trigger: done, then GET /browse/job/:uid for the final fragment.  htmx itself is not
// shipped (air-gapped servers): this file does the three swaps it would do.
async function post(url, form){
  const h = hdrs(); delete h['Content-Type'];
  return fetch(url, {method:'POST', headers:h, body: form || null});
}
async function search(){
  const fd = new FormData(); fd.append('search', document.getElementById('q').value);
  const r = await post('/browse/search/models', fd);
  document.getElementById('cards').innerHTML = await r.text(); wire();
}
async function act(btn, kind){
  // gallery ids come from third-party indexes: read back from a data-* attribute (server-escaped)
  const id = btn.dataset.id, box = btn.closest('.actions');
  if(kind === 'delete' && !confirm('Are you sure you wish to delete the model?')) return;
  const r = await post('/browse/' + kind + '/model/' + encodeURIComponent(id));
  box.innerHTML = await r.text(); poll(box);
}
function poll(box){
  const job = box.querySelector('[data-job]'); if(!job) return wire();
  const uid = job.dataset.job, bar = job.querySelector('.pbar');
  const tick = async () => {
    const r = await fetch('/browse/job/progress/' + uid, {headers:hdrs()});
    bar.innerHTML = await r.text();
    if(r.headers.get('HX-Trigger') === 'done'){
      box.innerHTML = await (await fetch('/browse/job/' + uid, {headers:hdrs()})).text(); wire(); return;
    }
    if(bar.querySelector('.err')) { wire(); return; }
    setTimeout(tick, 600);
  };
  tick();
}
function wire(){
  for(const b of document.querySelectorAll('button[data-act]')) b.onclick = () => act(b, b.dataset.act);
  for(const box of document.querySelectorAll('.actions')) if(box.querySelector('[data-job]') && !box.dataset.polling){
    box.dataset.polling = '1'; poll(box); }
}
window.addEventListener('load', wire);
"""

_TTS_JS = _AUTH_JS + """
async function speak(){
  const body = {model: document.getElementById('model').value, input: document.getElementById('txt').value};
  const v = document.getElementById('voice').value, b = document.getElementById('backend').value;
  if(v) body.voice = v; if(b) body.backend = b;
  const r = await fetch('/tts', {method:'POST', headers:hdrs(), body: JSON.stringify(body)});
  if(!r.ok){document.getElementById('st').textContent = 'error: ' + r.status + ' ' + await r.text(); return;}
  const a = document.getElementById('audio'); a.src = URL.createObjectURL(await r.blob()); a.play();
}
"""

_IMG_JS = _AUTH_JS + """
async function gen(){
  const st = document.getElementById('st'); st.textContent = 'generating...';
  // the reference's prompt syntax: "positive|negative"
  const neg = document.getElementById('neg').value.trim(), pos = document.getElementById('txt').value;
  const t0 = performance.now();
  const r = await fetch('/v1/images/generations', {method:'POST', headers:hdrs(), body: JSON.stringify({
    model: document.getElementById('model').value, prompt: neg ? pos + '|' + neg : pos,
    size: document.getElementById('size').value, step: parseInt(document.getElementById('steps').value) || undefined,
    seed: parseInt(document.getElementById('seed').value) || undefined, response_format: 'b64_json'})});
  if(!r.ok){st.textContent = 'error: ' + r.status + ' ' + await r.text(); return;}
  const j = await r.json(); st.textContent = ((performance.now() - t0) / 1000).toFixed(2) + ' s';
  const im = document.createElement('img'); im.src = 'data:image/png;base64,' + j.data[0].b64_json; im.title = pos;
  const g = document.getElementById('gallery'); g.insertBefore(im, g.firstChild);
}
"""

_SOUND_JS = _AUTH_JS + """
async function gen(){
  const st = document.getElementById('st'); st.textContent = 'generating...';
  const body = {model_id: document.getElementById('model').value, text: document.getElementById('txt').value};
  const d = parseFloat(document.getElementById('dur').value); if(d) body.duration_seconds = d;
  const r = await fetch('/v1/sound-generation', {method:'POST', headers:hdrs(), body: JSON.stringify(body)});
  if(!r.ok){st.textContent = 'error: ' + r.status + ' ' + await r.text(); return;}
  st.textContent = ''; const a = document.getElementById('audio'); a.src = URL.createObjectURL(await r.blob()); a.play();
}
"""

_HOME_JS = _AUTH_JS + """
async function unload(btn){
  await fetch('/backend/shutdown', {method:'POST', headers:hdrs(), body: JSON.stringify({model: btn.dataset.model})});
  location.reload();
}
async function monitor(btn){
  const r = await fetch('/backend/monitor?model=' + encodeURIComponent(btn.dataset.model), {headers:hdrs()});
  btn.closest('tr').querySelector('td.mon').textContent = r.ok ? JSON.stringify(await r.json()) : 'error ' + r.status;
}
"""

_TALK_JS = _AUTH_JS + """
// push-to-talk loop of the reference's /talk page (core/http/routes/ui.go talk route):
// microphone -> /v1/audio/transcriptions -> /v1/chat/completions -> /tts -> playback
let rec = null, chunks = [], history = [];
function val(id){ return document.getElementById(id).value; }
async function toggle(){
  const st = document.getElementById('st'), b = document.getElementById('rec');
  if(rec){ rec.stop(); b.textContent = 'Record'; return; }
  const stream = await navigator.mediaDevices.getUserMedia({audio:true});
  rec = new MediaRecorder(stream); chunks = [];
  rec.ondataavailable = e => chunks.push(e.data);
  rec.onstop = async () => {
    rec = null; stream.getTracks().forEach(t => t.stop());
    st.textContent = 'transcribing...';
    const fd = new FormData(); fd.append('file', new Blob(chunks, {type:'audio/webm'}), 'talk.webm');
    fd.append('model', val('whisper'));
    const h = hdrs(); delete h['Content-Type'];
    const tr = await fetch('/v1/audio/transcriptions', {method:'POST', headers:h, body:fd});
    if(!tr.ok){ st.textContent = 'transcription error: ' + tr.status; return; }
    const text = (await tr.json()).text || '';
    history.push({role:'user', content:text}); st.textContent = 'you: ' + text + ' / thinking...';
    const cr = await fetch('/v1/chat/completions', {method:'POST', headers:hdrs(), body: JSON.stringify({
      model: val('model'), messages: history})});
    if(!cr.ok){ st.textContent = 'chat error: ' + cr.status; return; }
    const reply = (await cr.json()).choices[0].message.content || '';
    history.push({role:'assistant', content:reply});
    document.getElementById('log').textContent += '> ' + text + '\\n' + reply + '\\n';
    const sp = await fetch('/tts', {method:'POST', headers:hdrs(), body: JSON.stringify({model: val('tts'), input: reply})});
    if(!sp.ok){ st.textContent = 'tts error: ' + sp.status; return; }
    const a = document.getElementById('audio'); a.src = URL.createObjectURL(await sp.blob()); a.play();
    st.textContent = '';
  };
  rec.start(); b.textContent = 'Stop';
}
"""


def _drop_bad(s: str) -> str:
    """DOM-id-safe gallery id (ui.go's dropBadChars: '@' -> '__')."""
    return s.replace("@", "__")


def _progress_bar(pct) -> str:
    p = max(0.0, min(100.0, float(pct or 0)))
    return (f"<div class=progress role=progressbar aria-valuemin=0 aria-valuemax=100 aria-valuenow={p:.0f}>"
            f"<div class=bar style='width:{p:.0f}%'></div></div><span class=muted>{p:.0f}%</span>")


def _start_progress(uid: str, text: str) -> str:
    u = html.escape(uid)
    return (f"<div data-job=\"{u}\" hx-trigger=done hx-get=\"/browse/job/{u}\" hx-swap=outerHTML>"
            f"<h4 role=status>{html.escape(text)}</h4><div class=pbar hx-get=\"/browse/job/progress/{u}\" "
            f"hx-trigger='every 600ms' hx-swap=innerHTML>{_progress_bar(0)}</div></div>")


def _action_button(kind: str, gid: str) -> str:
    label = {"install": "Install", "delete": "Delete", "reinstall": "Reinstall"}[kind]
    route = "delete" if kind == "delete" else "install"
    return (f"<button data-act={route} data-id=\"{html.escape(gid)}\" hx-post=\"/browse/{route}/model/"
            f"{html.escape(urllib.parse.quote(gid, safe='@'))}\">{label}</button>")


def _model_cards(models, installed, processing: dict, statuses) -> str:
    """The gallery card list (elements.ListModels): name, description, repository, license, tags,
    links, and an action box holding the install / delete button or a running job's progress."""
    out = []
    for m in models:
        gname = (m.get("gallery") or {}).get("name", "")
        name = m.get("name", "")
        gid = f"{gname}@{name}"
        meta = [f"repository: {html.escape(gname)}"]
        if m.get("license"):
            meta.append(f"license: {html.escape(str(m['license']))}")
        tags = " ".join(f"<span class=tag>{html.escape(str(t))}</span>" for t in (m.get("tags") or []))
        links = " ".join(f"<a href=\"{html.escape(str(u))}\" target=_blank rel=noopener>link #{i + 1}</a>"
                         for i, u in enumerate(m.get("urls") or []))
        uid = processing.get(gid)
        if uid:
            st = statuses(uid) or {}
            box = _start_progress(uid, "Deletion" if st.get("deletion") else "Installation")
        elif name in installed:
            box = _action_button("reinstall", gid) + " " + _action_button("delete", gid)
        else:
            box = _action_button("install", gid)
        out.append(f"<div class=card><h4>{html.escape(name)}</h4><p class=muted>"
                   f"{html.escape((m.get('description') or '')[:300])}</p><p class=muted>{' · '.join(meta)}</p>"
                   f"<p>{tags}</p><p>{links}</p><div class=actions id=\"action-div-{html.escape(_drop_bad(gid))}\">"
                   f"{box}</div></div>")
    return "".join(out) or "<p class=muted>no models match</p>"


def _search(models, term: str):
    """GalleryModels.Search (core/gallery/request.go:39-51): case-sensitive substring of the name,
    the description, the gallery name or the comma-joined tags."""
    return [m for m in models if term in m.get("name", "") or term in (m.get("description") or "")
            or term in (m.get("gallery") or {}).get("name", "") or term in ",".join(m.get("tags") or [])]


def build_router(state) -> APIRouter:
    r = APIRouter()

    def models():
        return state.list_models()

    async def home(request: Request):
        if state.cfg.disable_webui or "text/html" not in request.headers.get("accept", ""):
            return JSONResponse({"version": __version__, "models": models(),
                                 "loaded": [m.id for m in state.manager.list_loaded()],
                                 "uptime_s": round(time.time() - state.start_time, 1)})
        loaded = {m.id: m for m in state.manager.list_loaded()}

        def row(m):
            q = html.escape(urllib.parse.quote(m, safe=""))
            lm = loaded.get(m)
            acts = (f"<a href='/chat/{q}'>chat</a> · <a href='/tts/{q}'>tts</a> · <a href='/text2image/{q}'>image</a>")
            if lm is not None:
                acts += (f" · <button data-model=\"{html.escape(m)}\" onclick='monitor(this)'>monitor</button>"
                         f" <button data-model=\"{html.escape(m)}\" onclick='unload(this)'>unload</button>")
            state_ = f"loaded ({html.escape(lm.backend_name)})" if lm is not None else ""
            return f"<tr><td>{html.escape(m)}</td><td>{state_}</td><td>{acts}</td><td class='mon muted'></td></tr>"
        rows = "".join(row(m) for m in models())
        body = (f"<h2>Installed models</h2><table><thead><tr><th>model</th><th>state</th><th></th><th></th></tr></thead>"
                f"<tbody>{rows or '<tr><td colspan=4 class=muted>no models yet: install one from the gallery</td></tr>'}"
                f"</tbody></table><p class=muted>version {html.escape(__version__)} · "
                f"<a href='/metrics'>metrics</a> · <a href='/system'>system</a> · <a href='/swagger'>API docs</a></p>")
        return _page("LocalAI", body, _HOME_JS)

    # gallery id -> job uid of the install / delete running from the UI (ui.go processingModels)
    processing: dict = {}

    async def _available():
        import asyncio

        from .. import gallery as gal
        return [m.to_json() for m in await asyncio.to_thread(gal.available_models, state.cfg.galleries,
                                                              state.models_path)]

    def _status(uid):
        g = getattr(state, "gallery", None)
        return g.get(uid) if g is not None else None

    async def browse():
        try:
            avail, err = await _available(), ""
        except Exception as e:  # gallery unreachable (air-gapped): show installed only
            avail, err = [], str(e)
        cards = _model_cards(avail, set(models()), processing, _status)
        body = ("<h2>Model gallery</h2><div class=row><input id=q name=search placeholder='search' "
                "hx-post=/browse/search/models hx-trigger='keyup changed delay:500ms' hx-target=#cards "
                "oninput='search()'></div>"
                + (f"<p class=muted>gallery unavailable: {html.escape(err)}</p>" if err else "")
                + f"<p class=muted>{len(avail)} models available</p><div id=cards>{cards}</div>")
        return _page("Models", body, _BROWSE_JS)

    async def browse_search(request: Request):
        from ..utils.multipart import read_form
        try:
            form = await read_form(request) if await request.body() else {}
        except ValueError:
            form = {}
        term = str(form.get("search", ""))
        try:
            avail = await _available()
        except Exception as e:
            return HTMLResponse(f"<p class=muted>gallery unavailable: {html.escape(str(e))}</p>")
        return HTMLResponse(_model_cards(_search(avail, term), set(models()), processing, _status))

    def _svc():
        g = getattr(state, "gallery", None)
        if g is None:
            raise RuntimeError("gallery service not running")
        return g

    async def browse_install(gid: str):
        from .. import gallery as gal
        op = gal.GalleryOp(id=gal.new_op_id(), gallery_model_name=gid, galleries=list(state.cfg.galleries))
        processing[gid] = op.id
        _svc().submit(op)
        return HTMLResponse(_start_progress(op.id, "Installation"))

    async def browse_delete(gid: str):
        from .. import gallery as gal
        name = gid.split("@", 1)[1] if "@" in gid else gid  # local models need no repository id
        op = gal.GalleryOp(id=gal.new_op_id(), gallery_model_name=name, delete=True)
        processing[name] = op.id
        processing[gid] = op.id
        _svc().submit(op)
        state.configs.remove(name)
        return HTMLResponse(_start_progress(op.id, "Deletion"))

    def _forget(uid: str):
        for k in [k for k, v in processing.items() if v == uid]:
            del processing[k]

    async def browse_job_progress(uid: str):
        st = _status(uid)
        if st is None:
            return HTMLResponse(_progress_bar(0))
        if st.get("error"):
            _forget(uid)
            name = st.get("gallery_model_name", "")
            return HTMLResponse(f"<div class=err><h4 role=status>Error {html.escape(str(st['error']))}</h4>"
                                f"{_action_button('install', name)}</div>")
        if st.get("processed") and float(st.get("progress") or 0) >= 100:
            return HTMLResponse(_progress_bar(100), headers={"HX-Trigger": "done"})
        return HTMLResponse(_progress_bar(st.get("progress", 0)))

    async def browse_job(uid: str):
        st = _status(uid) or {}
        gid = next((k for k, v in processing.items() if v == uid and "@" in k), "") or st.get("gallery_model_name", "")
        _forget(uid)
        if st.get("deletion"):
            return HTMLResponse(f"<h4 role=status>Deletion completed</h4>{_action_button('reinstall', gid)}")
        return HTMLResponse(f"<h4 role=status>Installation completed</h4>{_action_button('delete', gid)}")

    async def chat(model: str = ""):
        ms = models()
        model = model or (ms[0] if ms else "")
        body = (f"<h2>Chat</h2><div class=row>{_model_select(ms, model)}"
                f"<label>temperature</label><input id=temp type=number step=0.1 value=0.7 style='max-width:80px'>"
                f"<label>top_p</label><input id=topp type=number step=0.05 placeholder=default style='max-width:80px'>"
                f"<label>max tokens</label><input id=maxt type=number step=1 placeholder=default style='max-width:90px'>"
                f"<button onclick='clearChat()'>Clear</button></div>"
                f"<div class=row><input id=sys placeholder='system prompt (optional)'></div>"
                f"<div id=log></div><div class=row><textarea id=msg rows=3 placeholder='message (Enter to send)'>"
                f"</textarea><button onclick='send()'>Send</button></div>"
                f"<div class=row><label>attach image (vision models)</label><input id=img type=file accept='image/*'></div>"
                f"<div id=stats class=muted></div>")
        return _page("Chat", body, _CHAT_JS)

    async def chat_model(model: str):
        return await chat(model)

    async def tts(model: str = ""):
        ms = models()
        body = (f"<h2>Text to speech</h2><div class=row>{_model_select(ms, model or (ms[0] if ms else ''))}"
                f"<input id=voice placeholder='voice (optional)'><input id=backend placeholder='backend (optional)'></div>"
                f"<div class=row><textarea id=txt rows=3></textarea><button onclick='speak()'>Speak</button></div>"
                f"<audio id=audio controls></audio><div id=st class=muted></div>")
        return _page("TTS", body, _TTS_JS)

    async def tts_model(model: str):
        return await tts(model)

    async def text2image(model: str = ""):
        ms = models()
        sizes = "".join(f"<option>{z}</option>" for z in ("512x512", "256x256", "768x768", "1024x1024", "768x512",
                                                          "512x768"))
        body = (f"<h2>Text to image</h2><div class=row>{_model_select(ms, model or (ms[0] if ms else ''))}"
                f"<select id=size>{sizes}</select><label>steps</label>"
                f"<input id=steps type=number value=20 style='max-width:70px'><label>seed</label>"
                f"<input id=seed type=number placeholder=random style='max-width:100px'></div>"
                f"<div class=row><input id=txt placeholder=prompt><button onclick='gen()'>Generate</button></div>"
                f"<div class=row><input id=neg placeholder='negative prompt (optional)'></div>"
                f"<div id=st class=muted></div><div id=gallery class=grid></div>")
        return _page("Text to image", body, _IMG_JS)

    async def text2image_model(model: str):
        return await text2image(model)

    async def sound(model: str = ""):
        ms = models()
        body = (f"<h2>Sound generation</h2><div class=row>{_model_select(ms, model or (ms[0] if ms else ''))}"
                f"<label>seconds</label><input id=dur type=number step=0.5 placeholder=default style='max-width:90px'>"
                f"</div><div class=row><input id=txt placeholder='describe the sound or music'>"
                f"<button onclick='gen()'>Generate</button></div><audio id=audio controls></audio>"
                f"<div id=st class=muted></div>")
        return _page("Sound generation", body, _SOUND_JS)

    async def sound_model(model: str):
        return await sound(model)

    async def talk():
        ms = models()
        first = ms[0] if ms else ""
        sel = [_model_select(ms, first, k) for k in ("model", "whisper", "tts")]
        body = ("<h2>Talk</h2><div class=row><label>LLM</label>" + sel[0] + "<label>whisper</label>" + sel[1]
                + "<label>tts</label>" + sel[2] + "</div><div class=row><button id=rec onclick='toggle()'>Record"
                "</button></div><pre id=log></pre><audio id=audio controls></audio><div id=st class=muted></div>")
        return _page("Talk", body, _TALK_JS)

    r.add_api_route("/", home, methods=["GET"])
    if not state.cfg.disable_webui:
        r.add_api_route("/browse", browse, methods=["GET"])
        r.add_api_route("/browse/search/models", browse_search, methods=["POST"])
        r.add_api_route("/browse/install/model/{gid:path}", browse_install, methods=["POST"])
        r.add_api_route("/browse/delete/model/{gid:path}", browse_delete, methods=["POST"])
        r.add_api_route("/browse/job/progress/{uid}", browse_job_progress, methods=["GET"])
        r.add_api_route("/browse/job/{uid}", browse_job, methods=["GET"])
        r.add_api_route("/chat/", chat, methods=["GET"])
        r.add_api_route("/chat/{model}", chat_model, methods=["GET"])
        r.add_api_route("/tts/", tts, methods=["GET"])
        r.add_api_route("/tts/{model}", tts_model, methods=["GET"])
        r.add_api_route("/text2image/", text2image, methods=["GET"])
        r.add_api_route("/text2image/{model}", text2image_model, methods=["GET"])
        r.add_api_route("/talk/", talk, methods=["GET"])
        r.add_api_route("/sound/", sound, methods=["GET"])
        r.add_api_route("/sound/{model}", sound_model, methods=["GET"])
    return r

