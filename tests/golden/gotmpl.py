"""Minimal, independent re-implementation of the parts of Go's ``text/template``
and ``sigs.k8s.io/yaml.YAMLToJSON`` that kwok's ``renderer.renderToJSON``
(reference: pkg/kwok/controllers/renderer.go:49-89) exercises.

This is fixture-generation tooling only (it never ships to the GPU box and is
never imported by the product).  It lets ``make_golden.py`` execute the
reference's *own* template files (pkg/kwok/controllers/templates/*.tpl, read
from /root/reference at generation time) so that the golden byte vectors are
pinned by the reference's templates rather than by our restatement of them.

Covered subset of text/template (Go 1.19 semantics):
  * text / ``{{ pipeline }}`` actions, ``{{-`` / ``-}}`` trim markers
  * ``with``/``else``/``end``, ``range``/``else``/``end``, ``if``/``else``/``end``
  * ``$v := pipeline`` declarations, ``$v`` and ``$`` references
  * field chains ``.a.b`` on maps (missing key -> "no value")
  * function calls with literal / dot / field / variable arguments
  * ``truth`` (template/exec.go isTrue): nil, false, 0, "" and empty
    map/slice are false
  * printing: strings verbatim, nil -> ``<no value>``

YAML -> JSON follows yaml.v2 (YAML 1.1) typing of plain scalars as used by
sigs.k8s.io/yaml v1.3.0: bools (y/yes/on/true/...), null (~/null), ints,
floats; *timestamps stay strings* (yaml.v2 decode.go keeps the original text
for timestamp-tagged scalars decoded into interface{}).  JSON output follows
encoding/json.Marshal of map[string]interface{}: sorted keys, compact, HTML
escaping of <, >, & and U+2028/U+2029.
"""
from __future__ import annotations

import json
import re

import yaml

NO_VALUE = object()  # Go's "<no value>" (nil interface / missing map key)


# ----------------------------------------------------------------------------
# lexer / parser
# ----------------------------------------------------------------------------
class _Text:
    def __init__(self, s):
        self.s = s


class _Action:
    def __init__(self, pipe):
        self.pipe = pipe


class _Block:
    def __init__(self, kind, pipe):
        self.kind = kind  # "with" | "range" | "if"
        self.pipe = pipe
        self.body = []
        self.else_body = None


_TOKEN_RE = re.compile(
    r'\s*(?:(?P<decl>:=)|(?P<str>"(?:[^"\\]|\\.)*")|(?P<num>-?\d+(?:\.\d+)?)'
    r'|(?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)'
    r'|(?P<field>(?:\.[A-Za-z0-9_]+)+|\.)|(?P<ident>[A-Za-z_][A-Za-z0-9_]*))'
)


def _tokenize(src):
    out = []
    pos = 0
    src = src.strip()
    while pos < len(src):
        m = _TOKEN_RE.match(src, pos)
        if not m or m.end() == pos:
            raise ValueError("cannot tokenize action: %r at %d" % (src, pos))
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        pos = m.end()
    return out


def parse(text):
    """Parse template text into a node list."""
    nodes = []
    stack = [nodes]
    blocks = []
    pos = 0
    while True:
        i = text.find("{{", pos)
        if i < 0:
            stack[-1].append(_Text(text[pos:]))
            break
        j = text.find("}}", i)
        if j < 0:
            raise ValueError("unclosed action")
        pre = text[pos:i]
        inner = text[i + 2 : j]
        pos = j + 2
        if inner.startswith("- "):
            pre = pre.rstrip(" \t\r\n")
            inner = inner[2:]
        if inner.endswith(" -"):
            inner = inner[:-2]
            # trim leading whitespace of following text
            k = pos
            while k < len(text) and text[k] in " \t\r\n":
                k += 1
            pos = k
        if pre:
            stack[-1].append(_Text(pre))
        toks = _tokenize(inner)
        if not toks:
            raise ValueError("empty action")
        head = toks[0]
        if head == ("ident", "end"):
            stack.pop()
            blocks.pop()
        elif head == ("ident", "else"):
            b = blocks[-1]
            b.else_body = []
            stack[-1] = b.else_body
        elif head[0] == "ident" and head[1] in ("with", "range", "if"):
            b = _Block(head[1], toks[1:])
            stack[-1].append(b)
            blocks.append(b)
            stack.append(b.body)
        else:
            stack[-1].append(_Action(toks))
    if blocks:
        raise ValueError("unterminated block")
    return nodes


# ----------------------------------------------------------------------------
# evaluation
# ----------------------------------------------------------------------------
def is_true(v):
    """template/exec.go isTrue for the JSON-decoded value domain."""
    if v is NO_VALUE or v is None:
        return False
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return v != 0
    if isinstance(v, (str, list, dict)):
        return len(v) != 0
    return True


def _field(v, path):
    for name in path.split(".")[1:]:
        if not name:
            continue
        if isinstance(v, dict):
            v = v.get(name, NO_VALUE)
        else:
            # Go: nil pointer evaluating interface {}.name -> error; our
            # inputs never do this.
            raise ValueError("field %s of non-map %r" % (name, v))
    return v


class GoNumber(str):
    """json.Number (decoder.UseNumber): printed verbatim."""


def _operand(tok, dot, scope, funcs):
    kind, val = tok
    if kind == "field":
        return dot if val == "." else _field(dot, val)
    if kind == "var":
        name, _, rest = val.partition(".")
        base = scope[name]
        return _field(base, "." + rest) if rest else base
    if kind == "num":
        return int(val) if re.fullmatch(r"-?\d+", val) else float(val)
    if kind == "str":
        return json.loads(val)
    if kind == "ident":
        return funcs[val]()
    raise ValueError(tok)


def _eval_pipe(toks, dot, scope, funcs):
    decl = None
    if len(toks) >= 2 and toks[1][0] == "decl":
        decl = toks[0][1]
        toks = toks[2:]
    head = toks[0]
    if head[0] == "ident" and len(toks) > 1:
        args = [_operand(t, dot, scope, funcs) for t in toks[1:]]
        v = funcs[head[1]](*args)
    else:
        if len(toks) != 1:
            raise ValueError("unsupported pipeline %r" % (toks,))
        v = _operand(head, dot, scope, funcs)
    if decl is not None:
        scope[decl] = v
        return None, True
    return v, False


def _print(v):
    if v is NO_VALUE or v is None:
        return "<no value>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, str):
        return str(v)
    if isinstance(v, (int, float)):
        return repr(v)
    raise ValueError("printing composite values is outside the covered subset")


def _exec(nodes, dot, scope, funcs, out):
    for n in nodes:
        if isinstance(n, _Text):
            out.append(n.s)
        elif isinstance(n, _Action):
            v, was_decl = _eval_pipe(n.pipe, dot, scope, funcs)
            if not was_decl:
                out.append(_print(v))
        else:
            v, _ = _eval_pipe(n.pipe, dot, scope, funcs)
            if n.kind == "range":
                items = []
                if isinstance(v, list):
                    items = v
                elif isinstance(v, dict):
                    items = [v[k] for k in sorted(v)]
                if items:
                    for it in items:
                        _exec(n.body, it, scope, funcs, out)
                elif n.else_body is not None:
                    _exec(n.else_body, dot, scope, funcs, out)
            else:
                if is_true(v):
                    _exec(n.body, v if n.kind == "with" else dot, scope, funcs, out)
                elif n.else_body is not None:
                    _exec(n.else_body, dot, scope, funcs, out)


def execute(text, data, funcs):
    nodes = parse(text)
    out = []
    _exec(nodes, data, {"$": data}, funcs, out)
    return "".join(out)


# ----------------------------------------------------------------------------
# YAML (yaml.v2 / YAML 1.1 typing) -> JSON (encoding/json)
# ----------------------------------------------------------------------------
class _GoYAMLLoader(yaml.SafeLoader):
    """SafeLoader with yaml.v2's implicit typing: no timestamp resolution
    (timestamps stay strings), y/Y/n/N are bools as in YAML 1.1."""


_GoYAMLLoader.yaml_implicit_resolvers = {
    k: [(tag, rx) for tag, rx in v if tag != "tag:yaml.org,2002:timestamp"]
    for k, v in yaml.SafeLoader.yaml_implicit_resolvers.items()
}
_BOOL_RE = re.compile(
    r"^(?:y|Y|yes|Yes|YES|n|N|no|No|NO|true|True|TRUE|false|False|FALSE|on|On|ON|off|Off|OFF)$"
)
for _ch in "yYnNtTfFoO":
    _GoYAMLLoader.yaml_implicit_resolvers[_ch] = [
        (tag, rx)
        for tag, rx in _GoYAMLLoader.yaml_implicit_resolvers.get(_ch, [])
        if tag != "tag:yaml.org,2002:bool"
    ] + [("tag:yaml.org,2002:bool", _BOOL_RE)]


def _construct_bool(loader, node):
    return node.value in ("y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON")


_GoYAMLLoader.add_constructor("tag:yaml.org,2002:bool", _construct_bool)


def go_json(v):
    """encoding/json.Marshal of the JSON-able value tree."""
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        if v == int(v) and abs(v) < 1e21:
            return str(int(v))
        return repr(v)
    if isinstance(v, str):
        return go_json_string(v)
    if isinstance(v, list):
        return "[" + ",".join(go_json(x) for x in v) + "]"
    if isinstance(v, dict):
        keys = sorted(v, key=lambda s: s.encode("utf-8"))
        return "{" + ",".join(go_json_string(k) + ":" + go_json(v[k]) for k in keys) + "}"
    raise TypeError(type(v))


def go_json_string(s):
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def yaml_to_json(text):
    """sigs.k8s.io/yaml.YAMLToJSON."""
    obj = yaml.load(text, Loader=_GoYAMLLoader)
    return go_json(obj)


def yaml_marshal(obj, indent=0):
    """controller.go:42-54 "YAML" template func: sigs.k8s.io/yaml.Marshal then
    optional indentation.  Exact YAML text differs from yaml.v2's emitter in
    spacing, but it re-parses to the same value tree, which is all that
    reaches the JSON output."""
    data = yaml.safe_dump(obj, default_flow_style=False, sort_keys=True)
    if indent > 0:
        pad = " " * (indent * 2)
        data = ("\n" + data).replace("\n", "\n" + pad)
    return data


def render_to_json(text, data, funcs):
    """renderer.go:49-89 renderToJSON: TrimSpace, execute, YAMLToJSON."""
    allf = {"YAML": yaml_marshal}
    allf.update(funcs)
    rendered = execute(text.strip(), data, allf)
    return yaml_to_json(rendered)
