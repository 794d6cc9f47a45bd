#!/usr/bin/env python3
"""Stand-in for ``ssh [-o opt]... [-p port] host command`` in the remote-node tests: runs
``command`` with /bin/sh on this machine, as the "remote" node whose task state lives under
``$FAKE_SSH_STATE_ROOT`` (so client and node keep separate state roots)."""
import os
import subprocess
import sys

args = sys.argv[1:]
while args and args[0].startswith("-"):
    flag = args.pop(0)
    if flag in ("-o", "-p", "-i", "-l"):
        args.pop(0)
host, command = args[0], args[1]
env = dict(os.environ, TPI_STATE_ROOT=os.environ["FAKE_SSH_STATE_ROOT"], FAKE_SSH_HOST=host)
with open(os.path.join(os.environ["FAKE_SSH_STATE_ROOT"], "ssh.log"), "a") as log:
    log.write(host + " " + command.split(" -m ", 1)[-1].split(" ")[1] + "\n")
sys.exit(subprocess.call(["/bin/sh", "-c", command], env=env))
