"""Writes the OPL parser fixtures from the reference checkout (run in the build container, where
/root/reference exists; the GPU box never reads the reference):

  opl_full_example.opl   the input of internal/schema/parser_test.go:19-72 ("full example")
  opl_full_example.json  its expected AST, internal/schema/.snapshots/TestParser-suite=snapshots-full_example.json
                         (a map namespace -> relations, the JSON of ast.Relation)
  opl_lexer.json         the lexer inputs of internal/schema/lexer_test.go:10-76 with the token
                         strings .snapshots/TestLexer-suite=snapshots-<name>.json records for them,
                         and the inputs that must end in a lexing error

Both are data: one test input and the reference's recorded output for it."""
import json
import os
import re

REF = "/root/reference/internal/schema"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    src = open(os.path.join(REF, "parser_test.go")).read()
    m = re.search(r'\{"full example", `(.*?)`\}', src, re.S)
    assert m, "full example not found"
    with open(os.path.join(HERE, "opl_full_example.opl"), "w") as f:
        f.write(m.group(1))
    snap = json.load(open(os.path.join(REF, ".snapshots", "TestParser-suite=snapshots-full_example.json")))
    with open(os.path.join(HERE, "opl_full_example.json"), "w") as f:
        json.dump(snap, f, indent=1, sort_keys=True)
        f.write("\n")
    lsrc = open(os.path.join(REF, "lexer_test.go")).read()
    cases = []
    block = lsrc[lsrc.index("var lexableTestCases"):lsrc.index("func TestLexer")]
    found = re.findall(r'\{"([^"]+)", `(.*?)`\}', block, re.S) + [(n, "") for n in re.findall(r'\{"([^"]+)", ""\}', block)]
    for name, body in found:
        snapf = os.path.join(REF, ".snapshots", "TestLexer-suite=snapshots-%s.json" % name.replace(" ", "_"))
        cases.append({"name": name, "input": body, "tokens": json.load(open(snapf))})
    errs = [{"name": n, "input": i} for n, i in
            re.findall(r'\{"([^"]+)", "((?:[^"\\]|\\.)*)"\}', lsrc[lsrc.index("var lexingErrorTestCases"):
                                                             lsrc.index("var lexableTestCases")])]
    errs = [{"name": e["name"], "input": json.loads('"%s"' % e["input"])} for e in errs]
    with open(os.path.join(HERE, "opl_lexer.json"), "w") as f:
        json.dump({"lexable": cases, "errors": errs}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
