"""``dfs_cli`` — command-line front end (C51; reference dfs/client/src/bin/dfs_cli.rs).

Same global flags and subcommands as the reference::

    dfs_cli [-m MASTER[,MASTER..]] [--config-servers A,B] [--max-retries N]
            [--initial-backoff-ms MS] [--host-alias a=b ...] [--ca-cert F] [--domain-name D]
      ls | put SRC DEST [--ec-data K --ec-parity M] | get SRC DEST | inspect PATH
      rename SRC DEST | delete PATH | safe-mode get|enter|leave
      cluster info|add-server ID ADDR|remove-server ID | shuffle PREFIX
      benchmark write|read|stress-write ... | check-history [PATH] [--self-test]
      workload --history F [--ops --clients --key-space --rename-ratio]
      presign s3://bucket/key [--method GET|PUT|DELETE] [--expires S] [--endpoint URL]

Additions: ``delete`` (the reference's linearizability script calls it but the CLI lacks
it), P50 in benchmark output, ``--json`` for benchmark results, ``--hedge-delay-ms`` to
enable hedged reads from the CLI, and ``cluster up`` to launch a local cluster.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import grpc

from ..client import benchmark as B
from ..client import checker
from ..client.client import Client, DfsError
from ..client.workload import run_workload
from ..models import proto as pb
from ..s3.auth.sigv4 import MAX_PRESIGN_EXPIRES, generate_presigned_url
from ..utils.rpc import ChannelPool, rpc_details, with_scheme


def parse_s3_url(url: str) -> tuple[str, str]:
    if not url.startswith("s3://"):
        raise ValueError("URL must start with s3://")
    path = url[5:]
    if "/" not in path:
        raise ValueError("URL must contain a key (s3://bucket/key)")
    bucket, key = path.split("/", 1)
    if not bucket or not key:
        raise ValueError("Bucket and key must not be empty")
    return bucket, key


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="dfs_cli", description="DFS CLI. Automatically discovers the Leader Master "
                                                             "node and retries operations on failure.")
    ap.add_argument("-m", "--master", default="http://127.0.0.1:50051")
    ap.add_argument("--config-servers", default="", help="comma-separated config server addresses")
    ap.add_argument("--max-retries", type=int, default=5)
    ap.add_argument("--initial-backoff-ms", type=int, default=500)
    ap.add_argument("--host-alias", action="append", default=[],
                    help="map internal hostnames to local addresses (e.g. master1:50051=localhost:50051)")
    ap.add_argument("--ca-cert", help="CA certificate for TLS")
    ap.add_argument("--domain-name", help="domain name for TLS certificate verification")
    ap.add_argument("--hedge-delay-ms", type=int, default=None, help="enable hedged reads after this delay")
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("ls", help="list all files (all shards)")
    p = sub.add_parser("put", help="upload a local file")
    p.add_argument("source")
    p.add_argument("dest")
    p.add_argument("--ec-data", type=int, default=0)
    p.add_argument("--ec-parity", type=int, default=0)
    p = sub.add_parser("get", help="download a file")
    p.add_argument("source")
    p.add_argument("dest")
    p = sub.add_parser("inspect", help="show file metadata and block locations")
    p.add_argument("path")
    p = sub.add_parser("rename")
    p.add_argument("source")
    p.add_argument("dest")
    p = sub.add_parser("delete")
    p.add_argument("path")
    p = sub.add_parser("safe-mode")
    p.add_argument("action", choices=["get", "enter", "leave"])
    p = sub.add_parser("cluster")
    cs = p.add_subparsers(dest="action", required=True)
    cs.add_parser("info")
    a = cs.add_parser("add-server")
    a.add_argument("server_id", type=int)
    a.add_argument("server_address")
    a = cs.add_parser("remove-server")
    a.add_argument("server_id", type=int)
    a = cs.add_parser("up", help="launch a local cluster and block until Ctrl-C")
    a.add_argument("--chunkservers", type=int, default=3)
    a.add_argument("--gpus", default="", help="comma-separated GPU ids (one chunkserver per GPU)")
    a.add_argument("--shards", type=int, default=1)
    a.add_argument("--masters-per-shard", type=int, default=1)
    a.add_argument("--s3", action="store_true", help="also start the S3 gateway")
    a.add_argument("--base-dir")
    p = sub.add_parser("shuffle")
    p.add_argument("prefix")
    p = sub.add_parser("benchmark")
    bs = p.add_subparsers(dest="action", required=True)
    w = bs.add_parser("write")
    w.add_argument("-c", "--count", type=int, default=100)
    w.add_argument("-s", "--size", type=int, default=1048576)
    w.add_argument("-n", "--concurrency", type=int, default=10)
    w.add_argument("-p", "--prefix", default="bench_write")
    w.add_argument("--json", action="store_true")
    r = bs.add_parser("read")
    r.add_argument("-p", "--prefix", default="bench_write")
    r.add_argument("-n", "--concurrency", type=int, default=10)
    r.add_argument("--json", action="store_true")
    sw = bs.add_parser("stress-write")
    sw.add_argument("-d", "--duration", type=float, default=30)
    sw.add_argument("-s", "--size", type=int, default=1048576)
    sw.add_argument("-n", "--concurrency", type=int, default=10)
    sw.add_argument("-p", "--prefix", default="bench_stress")
    sw.add_argument("--json", action="store_true")
    p = sub.add_parser("check-history", help="check a JSONL history for linearizability")
    p.add_argument("path", nargs="?", default="")
    p.add_argument("--self-test", action="store_true")
    p = sub.add_parser("workload", help="run a concurrent workload and record its history")
    p.add_argument("--ops", type=int, default=50)
    p.add_argument("--clients", type=int, default=5)
    p.add_argument("--key-space", type=int, default=4)
    p.add_argument("--rename-ratio", type=float, default=0.3)
    p.add_argument("--history", required=True)
    p = sub.add_parser("presign", help="generate a pre-signed S3 URL")
    p.add_argument("url")
    p.add_argument("--method", default="GET")
    p.add_argument("--expires", type=int, default=3600)
    p.add_argument("--endpoint")
    return ap


def make_client(a) -> Client:
    masters = [m.strip() for m in a.master.split(",") if m.strip()]
    cfg = [c.strip() for c in a.config_servers.split(",") if c.strip()]
    c = Client(masters, cfg, max_retries=a.max_retries, initial_backoff_ms=a.initial_backoff_ms, ca_cert=a.ca_cert,
               domain_name=a.domain_name, hedge_delay_ms=a.hedge_delay_ms)
    for pair in a.host_alias:
        if "=" in pair:
            alias, real = pair.split("=", 1)
            c.add_host_alias(alias.strip(), real.strip())
    if cfg:
        try:
            c.refresh_shard_map()
        except (DfsError, grpc.RpcError) as e:
            print(f"warning: could not fetch shard map: {e}", file=sys.stderr)
    return c


def _master_call(a, method: str, req):
    """Direct call to the first --master (safe-mode / cluster admin RPCs, like the reference)."""
    pool = ChannelPool(a.ca_cert, a.domain_name)
    try:
        addr = with_scheme(a.master.split(",")[0].strip(), a.ca_cert is not None)
        return pool.call(addr, "MasterService", method, req, timeout=30.0)
    finally:
        pool.close()


def _print_stats(st: B.Stats, as_json: bool) -> None:
    if as_json:
        print(json.dumps({"name": st.name, **st.summary()}))
    else:
        print(st.format())


def cmd_presign(a) -> int:
    ak = os.environ.get("AWS_ACCESS_KEY_ID")
    sk = os.environ.get("AWS_SECRET_ACCESS_KEY")
    if not ak:
        print("AWS_ACCESS_KEY_ID environment variable not set", file=sys.stderr)
        return 1
    if not sk:
        print("AWS_SECRET_ACCESS_KEY environment variable not set", file=sys.stderr)
        return 1
    region = os.environ.get("AWS_REGION") or os.environ.get("AWS_DEFAULT_REGION") or "us-east-1"
    endpoint = a.endpoint or os.environ.get("S3_ENDPOINT") or "http://localhost:9000"
    try:
        bucket, key = parse_s3_url(a.url)
    except ValueError as e:
        print(str(e), file=sys.stderr)
        return 1
    method = a.method.upper()
    if method not in ("GET", "PUT", "DELETE"):
        print(f"Unsupported method '{a.method}'. Supported methods: GET, PUT, DELETE", file=sys.stderr)
        return 1
    if not 1 <= a.expires <= MAX_PRESIGN_EXPIRES:
        print(f"--expires must be between 1 and {MAX_PRESIGN_EXPIRES} seconds", file=sys.stderr)
        return 1
    print(generate_presigned_url(endpoint, bucket, key, method, ak, sk, region, a.expires))
    return 0


def cmd_cluster_up(a) -> int:
    from ..cluster.launcher import LocalCluster

    gpus = [int(g) for g in a.gpus.split(",") if g.strip()] or None
    c = LocalCluster(a.base_dir, n_chunkservers=a.chunkservers, gpus=gpus, shards=a.shards,
                     masters_per_shard=a.masters_per_shard).start()
    try:
        print(f"masters: {','.join(c.master_addrs)}")
        if c.config_addrs:
            print(f"config servers: {','.join(c.config_addrs)}")
        print(f"chunkservers: {','.join(c.cs_addrs)}")
        if a.s3:
            print(f"s3: {c.start_s3()}")
        print(f"data: {c.base}  (Ctrl-C to stop)", flush=True)
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        pass
    finally:
        c.stop()
    return 0


def run(a) -> int:
    if a.cmd == "presign":
        return cmd_presign(a)
    if a.cmd == "check-history":
        if a.self_test:
            failures = checker.run_self_tests()
            if failures:
                print("Checker self-test FAILED: " + "; ".join(failures), file=sys.stderr)
                return 1
            print("All checker self-tests passed.")
            return 0
        if not a.path:
            print("check-history needs a history file (or --self-test)", file=sys.stderr)
            return 1
        try:
            with open(a.path) as f:
                ops = checker.parse_history(f)
        except OSError as e:
            print(f"Cannot open {a.path}: {e}", file=sys.stderr)
            return 1
        except checker.HistoryError as e:
            print(f"Parse error: {e}", file=sys.stderr)
            return 1
        print(f"Parsed {len(ops)} operations")
        violations = checker.check_linearizability(ops)
        if violations:
            print("Linearizability FAILED:", file=sys.stderr)
            for v in violations:
                print(f"  - {v}", file=sys.stderr)
            return 1
        print("Linearizability check PASSED")
        return 0
    if a.cmd == "cluster" and a.action == "up":
        return cmd_cluster_up(a)
    if a.cmd == "safe-mode":
        if a.action == "get":
            r = _master_call(a, "GetSafeModeStatus", pb.GetSafeModeStatusRequest())
            print("Safe Mode Status:")
            print(f"  Active: {str(r.is_safe_mode).lower()}")
            print(f"  Manual: {str(r.is_manual).lower()}")
            print(f"  ChunkServers: {r.chunk_server_count}")
            print(f"  Blocks: {r.reported_blocks}/{r.expected_blocks}")
            print(f"  Threshold: {int(r.threshold * 100)}%")
            return 0
        enter = a.action == "enter"
        r = _master_call(a, "SetSafeMode", pb.SetSafeModeRequest(enter=enter))
        if r.success:
            print("Entered Safe Mode" if enter else "Left Safe Mode")
            return 0
        print(f"Failed to {'enter' if enter else 'leave'} Safe Mode: {r.error_message}")
        return 1
    if a.cmd == "cluster":
        if a.action == "info":
            r = _master_call(a, "GetClusterInfo", pb.GetClusterInfoRequest())
            print("Raft Cluster Info:")
            print(f"  Node ID: {r.node_id}")
            print(f"  Role: {r.role}")
            print(f"  Term: {r.current_term}")
            print(f"  Leader ID: {r.leader_id}")
            print(f"  Leader Address: {r.leader_address}")
            print(f"  Commit Index: {r.commit_index}")
            print(f"  Last Applied: {r.last_applied}")
            print(f"  Members ({len(r.members)}):")
            for m in r.members:
                print(f"    - [{m.server_id}] {m.address} {'(self)' if m.is_self else ''}")
            return 0
        if a.action == "add-server":
            r = _master_call(a, "AddRaftServer", pb.AddRaftServerRequest(server_id=a.server_id,
                                                                         server_address=a.server_address))
            ok_msg = f"Added server {a.server_id} ({a.server_address}) to cluster"
        else:
            r = _master_call(a, "RemoveRaftServer", pb.RemoveRaftServerRequest(server_id=a.server_id))
            ok_msg = f"Removed server {a.server_id} from cluster"
        if r.success:
            print(ok_msg)
            return 0
        print(f"Failed to {'add' if a.action == 'add-server' else 'remove'} server: {r.error_message}")
        if r.leader_hint:
            print(f"Leader hint: {r.leader_hint}")
        return 1

    c = make_client(a)
    try:
        if a.cmd == "ls":
            for f in c.list_all_files():
                print(f)
        elif a.cmd == "put":
            if a.ec_data > 0 and a.ec_parity > 0:
                c.create_file(a.source, a.dest, ec=(a.ec_data, a.ec_parity))
                print(f"File uploaded successfully with EC RS({a.ec_data},{a.ec_parity})")
            else:
                c.create_file(a.source, a.dest)
                print("File uploaded successfully with replication")
        elif a.cmd == "get":
            c.get_file(a.source, a.dest)
            print("File downloaded successfully")
        elif a.cmd == "inspect":
            m = c.get_file_info(a.path)
            if m is None:
                print(f"File not found: {a.path}")
                return 0
            print(f"File Metadata for: {m.path}")
            print(f"  Size: {m.size} bytes")
            print(f"  Storage: EC RS({m.ec_data_shards},{m.ec_parity_shards})" if m.ec_data_shards > 0
                  else "  Storage: Replicated")
            print(f"  Blocks: {len(m.blocks)}")
            for i, b in enumerate(m.blocks):
                if b.ec_data_shards > 0:
                    print(f"    Block {i}: ID={b.block_id}, Size={b.size}, EC=RS({b.ec_data_shards},"
                          f"{b.ec_parity_shards}), OriginalSize={b.original_size}, Shards={list(b.locations)}")
                else:
                    print(f"    Block {i}: ID={b.block_id}, Size={b.size}, Locations={list(b.locations)}")
        elif a.cmd == "rename":
            c.rename_file(a.source, a.dest)
            print(f"File renamed successfully: {a.source} -> {a.dest}")
        elif a.cmd == "delete":
            c.delete_file(a.path)
            print(f"File deleted: {a.path}")
        elif a.cmd == "shuffle":
            c.initiate_shuffle(a.prefix)
            print(f"Triggered background shuffling for prefix: {a.prefix}")
        elif a.cmd == "workload":
            run_workload(c, a.history, ops=a.ops, clients=a.clients, key_space=a.key_space,
                         rename_ratio=a.rename_ratio)
            print("Workload completed.")
        elif a.cmd == "benchmark":
            if a.action == "write":
                if not a.json:
                    print(f"🚀 Starting Write Benchmark: {a.count} files, {a.size} bytes each, "
                          f"concurrency={a.concurrency}")
                st, _ = B.bench_write(c, a.count, a.size, a.concurrency, a.prefix)
                _print_stats(st, a.json)
            elif a.action == "read":
                if not a.json:
                    print(f"🚀 Starting Read Benchmark: prefix={a.prefix}, concurrency={a.concurrency}")
                files = [f for f in c.list_all_files() if f.startswith(a.prefix) or
                         f.lstrip("/").startswith(a.prefix.lstrip("/"))]
                if not files:
                    print(f"No files found matching prefix: {a.prefix}")
                    return 0
                if not a.json:
                    print(f"Found {len(files)} files to read")
                _print_stats(B.bench_read(c, a.prefix, a.concurrency, files=files), a.json)
            else:
                if not a.json:
                    print(f"🔥 Starting Write Stress Test: duration={a.duration}s, size={a.size} bytes, "
                          f"concurrency={a.concurrency}")
                st = B.bench_stress_write(c, a.duration, a.size, a.concurrency, a.prefix)
                _print_stats(st, a.json)
                if st.errors and not a.json:
                    print(f"Errors: {st.errors}")
        return 0
    finally:
        c.close()


def main(argv: list[str] | None = None) -> int:
    a = build_parser().parse_args(argv)
    try:
        return run(a)
    except (DfsError, OSError, ValueError) as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    except grpc.RpcError as e:
        print(f"Error: {rpc_details(e)}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
