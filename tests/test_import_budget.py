"""``tpi apply`` start-up stays cheap: the first half of the apply->first-log metric is the
CLI's own interpreter start + imports (round 5 lost 28 ms to an eager import of the
object-store HTTP clients).  A ``cloud = "local"`` apply must not load
``http.client``, ``ssl``, ``xml.etree`` or ``email.utils``; a task naming an object store
still gets them (lazily)."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEAVY = ("http.client", "ssl", "xml.etree", "xml.etree.ElementTree", "email.utils",
         # OpenSSL's hash module, tar and ctypes: ~9 ms more of every start (round 6)
         "_hashlib", "tarfile", "ctypes", "secrets",
         # sysconfig (the extension suffix) and a thread pool for one resource: ~6 ms (round 6)
         "sysconfig", "concurrent.futures")
# imported only once the task has started (its `addresses` attribute), not before: the
# rendezvous port is probed by the supervisor, not by `tpi apply` (round 6)
BEFORE_START = ("socket",)

MAIN_TF = '''
resource "iterative_task" "imports" {
  name    = "imports"
  cloud   = "local"
  storage {
    workdir = "."
  }
  script = <<-END
    #!/bin/sh
    echo "first log line"
  END
}
'''

PROBE = textwrap.dedent('''
    import atexit, json, os, sys
    sys.path.insert(0, %(root)r)
    out = %(out)r

    def dump():
        with open(out, "w") as f:
            json.dump(sorted(sys.modules), f)

    atexit.register(dump)
    from terraform_provider_iterative_amd.backends import node
    real_start = node.NodeTask.start

    def start(self, *a, **kw):  # what the CLI had loaded when it started the supervisor
        with open(out + ".start", "w") as f:
            json.dump(sorted(sys.modules), f)
        return real_start(self, *a, **kw)

    node.NodeTask.start = start
    sys.argv = ["tpi", "apply", "-auto-approve"]
    from terraform_provider_iterative_amd.cli.tf import main
    code = main()
    dump()
    os._exit(code or 0)
''')


def _apply_modules(tmp_path):
    from terraform_provider_iterative_amd import _build

    # the stamps' stat signatures current (a content check -- right after a checkout or an
    # edit of the sources -- imports the build's own modules once; not what is measured here)
    _build.build_native()
    _build.build_supervisor()
    work = tmp_path / "work"
    work.mkdir()
    (work / "main.tf").write_text(MAIN_TF)
    out = tmp_path / "modules.json"
    env = dict(os.environ, TPI_STATE_ROOT=str(tmp_path / "state"))
    try:
        proc = subprocess.run([sys.executable, "-c", PROBE % {"root": ROOT, "out": str(out)}],
                              cwd=work, env=env, capture_output=True, text=True, timeout=120)
        assert proc.returncode == 0, proc.stderr[-2000:]
        at_start = tmp_path / "modules.json.start"
        return set(json.loads(out.read_text())), set(json.loads(at_start.read_text()))
    finally:
        subprocess.run([sys.executable, os.path.join(ROOT, "bin", "tpi"), "destroy",
                        "-auto-approve"], cwd=work, env=env, capture_output=True, timeout=120)


def test_local_apply_does_not_import_the_object_store_clients(tmp_path):
    loaded, at_start = _apply_modules(tmp_path)
    assert "terraform_provider_iterative_amd.backends.node" in loaded  # the apply really ran
    assert not (loaded & set(HEAVY)), sorted(loaded & set(HEAVY))
    assert not (at_start & set(BEFORE_START)), sorted(at_start & set(BEFORE_START))
    assert "terraform_provider_iterative_amd.storage.objectstore" not in loaded


def test_object_store_names_parse_without_the_clients():
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from terraform_provider_iterative_amd.storage import remote\n"
            "assert remote.is_remote('s3://bucket/prefix')\n"
            "conn = remote.parse('gs://bucket/a', 'b')\n"
            "assert (conn.backend, conn.container, conn.path) == ('googlecloudstorage', 'bucket', 'a/b')\n"
            "assert remote.describe(conn) == 'gs://bucket/a/b'\n"
            "assert 'http.client' not in sys.modules and 'ssl' not in sys.modules\n"
            "r = remote.open_remote(remote.parse('s3://bucket', '', {'region': 'us-east-1'}))\n"
            "assert 'http.client' in sys.modules and type(r).__name__ == 'S3Remote'\n" % ROOT)
    proc = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=60)
    assert proc.returncode == 0, proc.stderr[-2000:]
