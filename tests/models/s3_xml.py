"""S3 XML bodies (C58; reference dfs/s3_server/src/s3_types.rs).

Element names and nesting follow the reference's quick-xml serialisation (no XML
namespace attribute, no declaration except on auth errors). Requests (multi-delete,
complete-multipart) are parsed namespace-agnostically so AWS SDK bodies with
``xmlns="http://s3.amazonaws.com/doc/2006-03-01/"`` are accepted too.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET
from xml.sax.saxutils import escape


def _el(tag: str, value) -> str:
    if value is None:
        return ""
    if isinstance(value, bool):
        value = "true" if value else "false"
    return f"<{tag}>{escape(str(value))}</{tag}>"


OWNER = "<Owner><ID>dfs</ID><DisplayName>dfs</DisplayName></Owner>"


def list_all_my_buckets(buckets: list[tuple[str, str]]) -> str:
    inner = "".join(f"<Bucket>{_el('Name', n)}{_el('CreationDate', d)}</Bucket>" for n, d in buckets)
    return f"<ListAllMyBucketsResult>{OWNER}<Buckets>{inner}</Buckets></ListAllMyBucketsResult>"


def _object(o: dict) -> str:
    return (f"<Contents>{_el('Key', o['key'])}{_el('LastModified', o['last_modified'])}{_el('ETag', o['etag'])}"
            f"{_el('Size', o['size'])}{_el('StorageClass', 'STANDARD')}{OWNER}</Contents>")


def _prefixes(cps: list[str]) -> str:
    return "".join(f"<CommonPrefixes>{_el('Prefix', p)}</CommonPrefixes>" for p in cps)


def list_bucket_v1(name: str, prefix: str, objects: list[dict], common_prefixes: list[str], marker: str = "",
                   max_keys: int = 1000, truncated: bool = False, next_marker: str | None = None) -> str:
    return (f"<ListBucketResult>{_el('Name', name)}{_el('Prefix', prefix)}{_el('Marker', marker)}"
            f"{_el('NextMarker', next_marker)}{_el('MaxKeys', max_keys)}{_el('IsTruncated', truncated)}"
            f"{''.join(_object(o) for o in objects)}{_prefixes(common_prefixes)}</ListBucketResult>")


def list_bucket_v2(name: str, prefix: str, objects: list[dict], common_prefixes: list[str], max_keys: int,
                   truncated: bool, key_count: int, continuation_token: str | None,
                   next_continuation_token: str | None, start_after: str | None) -> str:
    return (f"<ListBucketResult>{_el('Name', name)}{_el('Prefix', prefix)}{_el('MaxKeys', max_keys)}"
            f"{_el('IsTruncated', truncated)}{''.join(_object(o) for o in objects)}{_prefixes(common_prefixes)}"
            f"{_el('KeyCount', key_count)}{_el('ContinuationToken', continuation_token)}"
            f"{_el('NextContinuationToken', next_continuation_token)}{_el('StartAfter', start_after)}"
            "</ListBucketResult>")


def error(code: str, message: str, resource: str = "", request_id: str = "", **extra) -> str:
    more = "".join(_el(k, v) for k, v in extra.items())
    return (f"<Error>{_el('Code', code)}{_el('Message', message)}{_el('Resource', resource)}"
            f"{_el('RequestId', request_id)}{more}</Error>")


def initiate_mpu(bucket: str, key: str, upload_id: str) -> str:
    return (f"<InitiateMultipartUploadResult>{_el('Bucket', bucket)}{_el('Key', key)}{_el('UploadId', upload_id)}"
            "</InitiateMultipartUploadResult>")


def complete_mpu(location: str, bucket: str, key: str, etag: str) -> str:
    return (f"<CompleteMultipartUploadResult>{_el('Location', location)}{_el('Bucket', bucket)}{_el('Key', key)}"
            f"{_el('ETag', etag)}</CompleteMultipartUploadResult>")


def copy_object(last_modified: str, etag: str) -> str:
    return f"<CopyObjectResult>{_el('LastModified', last_modified)}{_el('ETag', etag)}</CopyObjectResult>"


def delete_result(deleted: list[str], errors: list[tuple[str, str, str]], quiet: bool = False) -> str:
    d = "" if quiet else "".join(f"<Deleted>{_el('Key', k)}</Deleted>" for k in deleted)
    e = "".join(f"<Error>{_el('Key', k)}{_el('Code', c)}{_el('Message', m)}</Error>" for k, c, m in errors)
    return f"<DeleteResult>{d}{e}</DeleteResult>"


def sts_result(access_key_id: str, secret: str, token: str, expiration: str, subject: str, role_id: str,
               arn: str) -> str:
    return ("<AssumeRoleWithWebIdentityResponse><AssumeRoleWithWebIdentityResult><Credentials>"
            f"{_el('AccessKeyId', access_key_id)}{_el('SecretAccessKey', secret)}{_el('SessionToken', token)}"
            f"{_el('Expiration', expiration)}</Credentials>{_el('SubjectFromWebIdentityToken', subject)}"
            f"<AssumedRoleUser>{_el('AssumedRoleId', role_id)}{_el('Arn', arn)}</AssumedRoleUser>"
            "</AssumeRoleWithWebIdentityResult></AssumeRoleWithWebIdentityResponse>")


def sts_error(code: str, message: str) -> str:
    return (f"<ErrorResponse><Error>{_el('Code', code)}{_el('Message', message)}</Error>"
            "<RequestId></RequestId></ErrorResponse>")


# ---------------------------------------------------------------------------- parsing
def _local(tag: str) -> str:
    return tag.rsplit("}", 1)[-1]


def _children(el, name: str):
    return [c for c in el if _local(c.tag) == name]


def _text(el, name: str, default: str | None = None) -> str | None:
    for c in el:
        if _local(c.tag) == name:
            return c.text or ""
    return default


def parse_delete_request(body: bytes) -> tuple[list[str], bool]:
    root = ET.fromstring(body)
    if _local(root.tag) != "Delete":
        raise ValueError("expected <Delete>")
    keys = [_text(o, "Key", "") for o in _children(root, "Object")]
    quiet = (_text(root, "Quiet", "false") or "false").strip().lower() == "true"
    return keys, quiet


def parse_complete_mpu(body: bytes) -> list[tuple[int, str]]:
    if not body.strip():
        return []
    root = ET.fromstring(body)
    return [(int(_text(p, "PartNumber", "0")), (_text(p, "ETag", "") or "").strip()) for p in _children(root, "Part")]


def parse(body: str | bytes) -> ET.Element:
    return ET.fromstring(body)


def find_text(el: ET.Element, path: list[str]) -> str | None:
    cur = el
    for name in path:
        nxt = next((c for c in cur if _local(c.tag) == name), None)
        if nxt is None:
            return None
        cur = nxt
    return cur.text
