"""Storage sync semantics (reference: task/common/machine/storage_test.go)."""
import os

import pytest

from terraform_provider_iterative_amd.storage import transfer as tr

REF_TREE = "/root/reference/task/common/machine/testdata/transferTest"


@pytest.fixture()
def transfer_tree(tmp_path):
    """The reference's transferTest tree (empty files; recreated so tests don't need it)."""
    root = tmp_path / "transferTest"
    (root / "temp").mkdir(parents=True)
    for rel in ("a.txt", "main.tf", "temp/a.txt", "temp/b.txt"):
        (root / rel).write_text("")
    if os.path.isdir(REF_TREE):
        assert sorted(_list(REF_TREE)) == sorted(_list(str(root)))
    return str(root)


def _list(d):
    out = []
    for base, dirs, files in os.walk(d):
        for name in dirs + files:
            out.append(os.path.join(base, name)[len(d):])
    return out


@pytest.mark.parametrize("exclude,expect", [
    (None, ["/a.txt", "/temp", "/temp/a.txt", "/temp/b.txt"]),  # builtin excludes drop main.tf
    (["**.txt"], ["/temp"]),                                   # directory still transferred
    (["/a.txt"], ["/temp", "/temp/a.txt", "/temp/b.txt"]),     # explicitly anchored
    (["a.txt"], ["/temp", "/temp/a.txt", "/temp/b.txt"]),      # implicitly anchored
])
def test_transfer_excludes(transfer_tree, tmp_path, exclude, expect):
    dst = str(tmp_path / "dst")
    tr.transfer(transfer_tree, dst, exclude)
    assert sorted(_list(dst)) == sorted(expect)


@pytest.mark.parametrize("conn,expected", [
    (tr.Connection("azureblob", "container", config={"account": "az_account", "key": "az_key"}),
     ":azureblob,account='az_account',key='az_key':container"),
    (tr.Connection("azureblob", "container", path="/subdirectory"), ":azureblob:container/subdirectory"),
    (tr.Connection("azureblob", "container", path="subdirectory"), ":azureblob:container/subdirectory"),
])
def test_connection_string(conn, expected):
    assert str(conn) == expected


def test_connection_parse_roundtrip():
    c = tr.Connection.parse(":local,a='1':/tmp/x")
    assert c.backend == "local" and c.config == {"a": "1"} and c.local_path() == "/tmp/x"
    assert tr.Connection.parse("/plain/dir").local_path() == "/plain/dir"
    with pytest.raises(NotImplementedError):
        tr.Connection.parse(":s3:bucket").local_path()


def test_limit_transfer(tmp_path):
    src = tmp_path / "src"
    for rel in ("results/epoch.txt", "results/sub/x.bin", "cache/big.bin", "top.txt",
                "results2/no.txt"):
        p = src / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(rel)
    rules = tr.limit_transfer("results", tr.transfer_rules(["cache"]))
    assert rules[-3:] == ["+ /results", "+ /results/**", "- /**"]
    dst = tmp_path / "dst"
    tr.transfer(str(src), str(dst), rules=rules)
    assert sorted(_list(str(dst))) == ["/results", "/results/epoch.txt", "/results/sub",
                                       "/results/sub/x.bin"]
    assert tr.limit_transfer(".", ["x"]) == ["x"]


def test_rule_translation():
    assert tr.transfer_rules(["a.txt", "dir/", "+ keep", "./x/../y"])[3:] == [
        "- /a.txt", "- /dir", "+ keep", "- /y"]


@pytest.mark.parametrize("glob,path,ok", [
    ("*.txt", "a.txt", True), ("*.txt", "d/a.txt", True), ("/*.txt", "d/a.txt", False),
    ("/**.txt", "d/e/a.txt", True), ("a?c", "abc", True), ("a?c", "a/c", False),
    ("[ab]x", "bx", True), ("[^ab]x", "bx", False), ("{foo,bar}.py", "x/bar.py", True),
    ("/dir/**", "dir/", True), ("/dir/**", "dirx/", False), ("\\*", "*", True),
])
def test_glob(native, glob, path, ok):
    assert native.glob_match(glob, path) is ok


def test_copy_is_incremental_and_preserves_metadata(tmp_path, native):
    src = tmp_path / "s"
    src.mkdir()
    f = src / "data.bin"
    f.write_bytes(os.urandom(300000))
    os.chmod(f, 0o640)
    os.utime(f, ns=(1_600_000_000_123_456_789, 1_600_000_000_123_456_789))
    (src / "empty").write_bytes(b"")
    dst = tmp_path / "d"
    flt = native.Filter([])
    first = native.copy_dir(str(src), str(dst), flt, 4, 4096)
    assert first["files"] == 2 and first["bytes"] == 300000
    assert (dst / "data.bin").read_bytes() == f.read_bytes()
    st = os.stat(dst / "data.bin")
    assert st.st_mtime_ns == 1_600_000_000_123_456_789 and (st.st_mode & 0o777) == 0o640
    second = native.copy_dir(str(src), str(dst), flt, 4, 4096)
    assert second["files"] == 0 and second["skipped"] == 2


def test_reports_and_status(tmp_path):
    rep = tmp_path / "reports"
    rep.mkdir()
    (rep / "task-1").write_text("2022-01-01T00:00:00Z hello\n")
    (rep / "status-1").write_text('{"result": "success", "code": "0", "status": "exited"}')
    (rep / "status-2").write_text('{"result": "exit-code", "code": "1", "status": "exited"}')
    (rep / "status-3").write_text('{"result": "timeout", "code": "", "status": "killed"}')
    assert tr.logs(str(tmp_path)) == ["2022-01-01T00:00:00Z hello\n"]
    assert tr.status(str(tmp_path), {"running": 2}) == {"running": 2, "succeeded": 1, "failed": 2}


def test_human_size():
    assert tr.human_size(0) == "0B"
    assert tr.human_size(1500) == "1.5kB"
    assert tr.human_size(10e9) == "10GB"


def test_existing_bucket_connection_strings():
    """Vectors of task/{aws,gcp}/resources/data_source_bucket_test.go."""
    aws = tr.Connection.existing_bucket(
        "aws", "pre-created-bucket", "subdirectory", {"region": "us-east-1"},
        {"AccessKeyID": "access-key-id", "SecretAccessKey": "secret-access-key",
         "SessionToken": "session-token"})
    assert str(aws) == (":s3,access_key_id='access-key-id',provider='AWS',region='us-east-1',"
                        "secret_access_key='secret-access-key',session_token='session-token'"
                        ":pre-created-bucket/subdirectory")
    gcp = tr.Connection.existing_bucket("gcp", "pre-created-bucket", "subdirectory",
                                        credentials={"ApplicationCredentials":
                                                     "gcp-credentials-json"})
    assert str(gcp) == (":googlecloudstorage,service_account_credentials='gcp-credentials-json'"
                        ":pre-created-bucket/subdirectory")
    az = tr.Connection.existing_bucket("az", "container", "sub",
                                       {"account": "a", "key": "k"})
    assert str(az) == ":azureblob,account='a',key='k':container/sub"


def test_link_tree_hard_links_with_the_transfer_filters(tmp_path):
    """TPI_PUSH_LINK=1's push: files become hard links (same inode, no bytes copied), the
    default excludes and user rules apply, and an existing target is replaced."""
    from terraform_provider_iterative_amd.storage.transfer import link_tree

    src, dst = tmp_path / "src", tmp_path / "dst"
    (src / "sub").mkdir(parents=True)
    (src / "train.py").write_text("print(1)\n")
    (src / "sub" / "data.bin").write_bytes(b"x" * 4096)
    (src / "main.tf").write_text("resource {}\n")          # default exclude
    (src / "skip.log").write_text("no\n")                  # user exclude
    (dst).mkdir()
    (dst / "train.py").write_text("stale\n")
    stats = link_tree(str(src), str(dst), ["skip.log"])
    assert stats["linked"] == 2 and stats["copied"] == 0 and stats["bytes"] == 4096 + 9
    assert os.stat(dst / "sub" / "data.bin").st_ino == os.stat(src / "sub" / "data.bin").st_ino
    assert (dst / "train.py").read_text() == "print(1)\n"
    assert not (dst / "main.tf").exists() and not (dst / "skip.log").exists()
