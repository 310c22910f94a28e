"""The subset of gin-config that Dopamine's .gin files use (gin is not installed
here; third-party, not vendored by the reference).

Supported: ``import ...`` lines (ignored: modules register what they provide),
``Configurable.param = value`` bindings (also module-qualified configurable
names, matched by suffix), Python literal values, ``%MACRO`` constants,
``@reference`` (the registered object) and ``@reference()`` (called, with its own
bindings applied), ``#`` comments and bracket/backslash line continuation.
Explicitly passed arguments win over bindings, as in gin.  Not supported: scopes
(``scope/Name.param``), macros or references nested inside container literals.
"""
import ast
import functools
import inspect
import re

_bindings = {}     # (configurable, param) -> parsed value
_constants = {}    # macro name -> value
_refs = {}         # reference name -> object


class _Macro(object):
  def __init__(self, name):
    self.name = name


class _Ref(object):
  def __init__(self, name, call):
    self.name, self.call = name, call


def constant(name, value):
  """gin.constant: makes ``%name`` resolve to ``value``."""
  _constants[name] = value


def register(name, obj):
  """Makes ``@name`` (and ``@name()``) resolve to ``obj``."""
  _refs[name] = obj
  return obj


def clear_config():
  _bindings.clear()


def _strip_comment(line):
  quote = None
  for i, ch in enumerate(line):
    if quote:
      if ch == quote:
        quote = None
    elif ch in '\'"':
      quote = ch
    elif ch == '#':
      return line[:i]
  return line


def _logical_lines(text):
  buf, depth = '', 0
  for raw in text.splitlines():
    line = _strip_comment(raw).rstrip()
    cont = line.endswith('\\')
    if cont:
      line = line[:-1]
    buf += (' ' if buf else '') + line.strip()
    depth += sum(line.count(c) for c in '([{') - sum(line.count(c) for c in ')]}')
    if cont or depth > 0:
      continue
    if buf:
      yield buf
    buf, depth = '', 0
  if buf:
    yield buf


def _parse_value(text):
  text = text.strip()
  if text.startswith('%'):
    return _Macro(text[1:].strip())
  if text.startswith('@'):
    name = text[1:].strip()
    call = name.endswith('()')
    return _Ref(name[:-2] if call else name, call)
  try:
    return ast.literal_eval(text)
  except (ValueError, SyntaxError):
    raise ValueError('Unsupported gin value: {!r}'.format(text))


_BINDING = re.compile(r'^([A-Za-z_][\w.]*)\.([A-Za-z_]\w*)\s*=\s*(.+)$')


def parse_config(text):
  for line in _logical_lines(text):
    if line.startswith('import ') or line.startswith('from '):
      continue
    m = _BINDING.match(line)
    if not m:
      raise ValueError('Unsupported gin statement: {!r}'.format(line))
    _bindings[(m.group(1), m.group(2))] = _parse_value(m.group(3))


def parse_config_files_and_bindings(config_files, bindings, skip_unknown=False):
  """gin.parse_config_files_and_bindings (run_experiment.py:40-51)."""
  del skip_unknown
  for f in config_files or []:
    with open(f) as fh:
      parse_config(fh.read())
  for b in bindings or []:
    parse_config(b)


def _matches(bound_name, name):
  return bound_name == name or bound_name.endswith('.' + name) or name.endswith('.' + bound_name)


def _lookup_ref(name):
  if name in _refs:
    return _refs[name]
  hits = [v for k, v in _refs.items() if _matches(k, name)]
  if len(hits) == 1:
    return hits[0]
  raise ValueError('Unknown gin reference @{}'.format(name))


def _resolve(v):
  if isinstance(v, _Macro):
    if v.name not in _constants:
      raise ValueError('Unknown gin macro %{}'.format(v.name))
    return _constants[v.name]
  if isinstance(v, _Ref):
    obj = _lookup_ref(v.name)
    return obj() if v.call else obj
  return v


def query(name):
  """{param: value} bound for the configurable ``name`` (resolved)."""
  return {p: _resolve(v) for (c, p), v in _bindings.items() if _matches(c, name)}


def configurable(name):
  """Decorator: missing keyword arguments of the wrapped callable are filled
  from the bindings of ``name`` (explicitly passed ones win)."""
  def deco(fn):
    sig = inspect.signature(fn)

    @functools.wraps(fn)
    def wrapped(*args, **kwargs):
      bound = sig.bind_partial(*args, **kwargs).arguments
      for p, v in query(name).items():
        if p not in bound:
          kwargs[p] = v
      return fn(*args, **kwargs)
    return wrapped
  return deco
