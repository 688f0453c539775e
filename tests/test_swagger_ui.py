"""The offline Swagger UI (assets/swagger-ui.html), the stand-in for the swagger-ui 2.1.4
webjar that the reference's landing page iframes (index.html:11-15). Its pure helpers run
under node against the served /api/swagger.json; the page itself is served by the server."""
import json
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PAGE = ROOT / "assets" / "swagger-ui.html"


def _node(js: str) -> object:
    node = shutil.which("node") or shutil.which("nodejs")
    if not node:
        pytest.skip("node is not installed")
    script = re.search(r"<script>\n(.*)</script>", PAGE.read_text(), re.S).group(1)
    prog = ("var module = {exports: {}};\n" + script + "\nvar S = module.exports;\n"
            "var spec = " + (ROOT / "assets" / "swagger.json").read_text() + ";\n"
            "process.stdout.write(JSON.stringify((function () {" + js + "})()));")
    r = subprocess.run([node, "-e", prog], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_operations_grouped_under_default_tag():
    """swagger-jaxrs emits no tags for HolaResource (no class-level @Api), so swagger-ui 2.x
    lists every operation under "default", the resource index.html deep-links to."""
    groups = _node("return S.groupOperations(spec).map(function (g) {"
                   "  return [g.tag, g.ops.map(function (o) { return [o.method, o.path, o.id]; })]; });")
    assert groups == [["default", [["get", "/hola", "hola"], ["get", "/hola-chaining", "holaChaining"],
                                   ["get", "/health", "health"]]]]


def test_models_urls_and_curl():
    out = _node("""
      var base = S.baseUrl(spec, 'http://h:8080/api/swagger.json', 'http://h:8080/webjars/swagger-ui/2.1.4/');
      return {
        base: base,
        models: [S.modelName(spec.paths['/hola'].get.responses['200'].schema),
                 S.modelName(spec.paths['/hola-chaining'].get.responses['200'].schema),
                 S.modelName({$ref: '#/definitions/Pet'})],
        url: S.requestUrl(base, '/hola', [], {}),
        q: S.requestUrl('http://x/api', '/p/{id}', [{name: 'id', in: 'path'}, {name: 'n', in: 'query'}],
                        {id: 'a b', n: '2'}),
        curl: S.curl('get', base + '/hola', S.headersFor([], {}, 'text/plain')),
        hash: [S.parseHash('#!/default'), S.parseHash('#!/default/hola'), S.parseHash('')],
        spec_url: S.specUrlFrom('?url=http%3A%2F%2Fh%2Fapi%2Fswagger.json', 'fallback'),
        json: S.prettyBody('["a","b"]', 'application/json'),
        empty: S.prettyBody('', 'text/plain'),
      };""")
    assert out["base"] == "http://h:8080/api"
    assert out["models"] == ["string", "Array[string]", "Pet"]
    assert out["url"] == "http://h:8080/api/hola"
    assert out["q"] == "http://x/api/p/a%20b?n=2"
    assert out["curl"] == "curl -X GET --header 'Accept: text/plain' 'http://h:8080/api/hola'"
    assert out["hash"] == [{"tag": "default", "op": None}, {"tag": "default", "op": "hola"}, None]
    assert out["spec_url"] == "http://h/api/swagger.json"
    assert out["json"] == '[\n  "a",\n  "b"\n]' and out["empty"] == "no content"


DOM_SHIM = """
  function Node(tag) {
    this.tagName = tag; this.children = []; this.style = {}; this.textContent = ''; this.id = '';
    var cls = {}; var self = this;
    this.classList = {add: function (c) { cls[c] = 1; }, remove: function (c) { delete cls[c]; },
                      toggle: function (c) { if (cls[c]) delete cls[c]; else cls[c] = 1; },
                      contains: function (c) { return !!cls[c]; }};
    Object.defineProperty(this, 'className', {set: function (v) { cls = {}; String(v).split(' ').forEach(function (c) { if (c) cls[c] = 1; }); },
                                               get: function () { return Object.keys(cls).join(' '); }});
  }
  Node.prototype.appendChild = function (c) { this.children.push(c); return c; };
  Node.prototype.all = function () {
    var out = [];
    this.children.forEach(function (c) { out.push(c); if (c.all) out = out.concat(c.all()); });
    return out;
  };
  Node.prototype.querySelectorAll = function (sel) {
    var c = sel.replace('.', '');
    return this.all().filter(function (n) { return n.classList && n.classList.contains(c); });
  };
  var roots = {info: new Node('div'), resources: new Node('div'), footer: new Node('div')};
  global.document = {
    createElement: function (t) { return new Node(t); },
    createTextNode: function (t) { var n = new Node('#text'); n.textContent = t; return n; },
    getElementById: function (id) {
      if (roots[id]) return roots[id];
      var all = roots.resources.all();
      for (var i = 0; i < all.length; ++i) if (all[i].id === id) return all[i];
      return null;
    }
  };
  global.window = {location: {hash: '#!/default/holaChaining', href: 'http://h:8080/webjars/swagger-ui/2.1.4/'}};
"""


def test_render_builds_the_page_and_honours_deep_links():
    """render() against a minimal DOM: one "default" resource with the three operations, the
    info block, the footer, and the #!/default/holaChaining deep link expanded."""
    out = _node(DOM_SHIM + """
      S.render(spec, 'http://h:8080/api/swagger.json');
      var ops = global.document.getElementById('resources').querySelectorAll('.op');
      return {
        ops: ops.map(function (o) { return [o.id, o.classList.contains('open')]; }),
        footer: global.document.getElementById('footer').textContent,
        title: global.document.getElementById('info').children[0].textContent,
      };""")
    assert out["ops"] == [["default_hola", False], ["default_holaChaining", True], ["default_health", False]]
    assert out["footer"] == "[ base url: /api , api version: 1.0.0 ]"
    assert out["title"] == "Hola microservices REST API"


def test_viewer_served_at_webjar_path(hola):
    s = hola()
    st, h, body = s.get("/webjars/swagger-ui/2.1.4/?url=http://x/api/swagger.json")
    assert st == 200 and h["content-type"].startswith("text/html")
    for label in (b"Try it out!", b"Response Content Type", b"Implementation Notes", b"Response Messages",
                  b"List Operations", b"Expand Operations", b"base url", b"Explore"):
        assert label in body, label
