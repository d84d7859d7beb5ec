"""The supported input domain as a table shared by the oracle
(CPU) and engine (GPU) tests: both must accept and reject exactly these.

A value a template renders with `{{ . }}` (container names / images,
readiness-gate types, nodeInfo fields) is inserted as a YAML plain scalar and
typed by gopkg.in/yaml.v2 v2.4.0 (resolve.go, [ext]) before encoding/json
emits it.  The engine emits it verbatim as a JSON string, so only values that
stay strings are in the domain.  IP strings follow Go 1.19 net.ParseIP for
IPv4 (leading zeros rejected since Go 1.17)."""

# (value, in domain?, reason)
STRINGS = [
    ("fake", True, "plain word"),
    ("nginx:1.25", True, "':' not followed by a space"),
    ("registry.io/org/img-3:v1.2_x@sha256", True, "image reference"),
    ("6.1.5", True, "not an int literal, not a yamlStyleFloat: stays a string"),
    ("5.15.0-1019-aws", True, "kernel version"),
    ("1abc", True, "digit-led but no number"),
    ("12:30", True, "yaml.v2 has no base-60 ints"),
    ("0x", True, "prefix without digits: ParseInt fails"),
    ("1e", True, "exponent without digits"),
    ("Ubuntu 22.04.3 LTS", True, "inner spaces stay in a plain scalar"),
    ("yes-please", True, "not a resolveMap word"),
    ("fake-pod", True, "default container name"),
    ("y", False, "bool (resolveMap)"),
    ("Yes", False, "bool"),
    ("on", False, "bool"),
    ("OFF", False, "bool"),
    ("null", False, "null"),
    ("Null", False, "null"),
    ("15", False, "int"),
    ("017", False, "octal int"),
    ("1_000", False, "int once '_' is removed"),
    ("0x1F", False, "hex int"),
    ("0b101", False, "binary int"),
    ("0o17", False, "octal int (0o)"),
    ("1.5", False, "float"),
    ("1e5", False, "float"),
    ("3.", False, "float (digits, dot)"),
    ("99999999999999999999", False, "out-of-range int reads as a float"),
    ("-x", False, "indicator first"),
    (".5", False, "not alnum first (a float anyway)"),
    ("a: b", False, "mapping indicator"),
    ("img:", False, "trailing ':'"),
    ("a ", False, "trailing space"),
    ("a#b", False, "character outside the domain"),
    ("a\"b", False, "character outside the domain"),
    ("", False, "empty"),
]

# values PyYAML's YAML 1.1 resolvers (the fixture generator, tests/golden/gotmpl.py)
# type differently from yaml.v2: base-60 ints, Go's 0o prefix, exponent
# floats without a dot
PYYAML_DIFFERS = {"12:30", "0o17", "1e5"}

# (dotted quad, in domain?)
IPS = [
    ("1.2.3.4", True),
    ("255.255.255.255", True),
    ("10.0.0.1", True),
    ("010.0.0.1", False),
    ("1.2.3.04", False),
    ("1.2.3.4.", False),
    ("1.2.3", False),
    ("256.1.1.1", False),
    ("1..2.3", False),
    ("0.0.0.0", False),
    ("::1", False),
    ("::ffff:1.2.3.4", False),
    (" 1.2.3.4", False),
]
