"""Minimal S3 client for ``s3://`` (and ``s3a://``/``s3n://``) paths: AWS Signature
Version 4 over plain HTTP(S), standard library only.

The reference reaches S3 through Hadoop's S3A file system (R10; Zs/common/Utils.scala
FS helpers take any Hadoop URI). This framework has no Hadoop client, so the object
operations the checkpoint / model-file paths need are implemented directly:
GET (optionally ranged), PUT, HEAD, DELETE and ListObjectsV2, with path-style
addressing against ``ZOO_S3_ENDPOINT`` / ``AWS_ENDPOINT_URL`` (S3-compatible stores,
MinIO, Ceph RGW) or ``https://s3.<region>.amazonaws.com``. Credentials come from
``AWS_ACCESS_KEY_ID`` / ``AWS_SECRET_ACCESS_KEY`` (/ ``AWS_SESSION_TOKEN``), the region
from ``AWS_REGION`` / ``AWS_DEFAULT_REGION`` (default us-east-1).
"""
import datetime
import hashlib
import hmac
import http.client
import os
import xml.etree.ElementTree as ET
from urllib.parse import quote, urlparse

EMPTY_SHA256 = hashlib.sha256(b"").hexdigest()


def _uri_encode(s, slash=True):
    return quote(s, safe="-_.~" + ("/" if slash else ""))


def _hmac(key, msg):
    return hmac.new(key, msg.encode("utf-8"), hashlib.sha256).digest()


def signing_key(secret, date, region, service="s3"):
    k = _hmac(("AWS4" + secret).encode("utf-8"), date)
    k = _hmac(k, region)
    k = _hmac(k, service)
    return _hmac(k, "aws4_request")


def sign_v4(method, canonical_uri, query, headers, payload_hash, access_key, secret, region, amz_date,
            service="s3"):
    """Return the Authorization header value. ``headers``: {name: value} INCLUDING host,
    x-amz-date and x-amz-content-sha256; ``query``: {name: value}; ``canonical_uri``: the
    already-encoded absolute path."""
    date = amz_date[:8]
    cq = "&".join("%s=%s" % (_uri_encode(k, False), _uri_encode(str(v), False)) for k, v in sorted(query.items()))
    hs = sorted((k.lower().strip(), " ".join(str(v).strip().split())) for k, v in headers.items())
    ch = "".join("%s:%s\n" % kv for kv in hs)
    sh = ";".join(k for k, _ in hs)
    creq = "\n".join([method, canonical_uri, cq, ch, sh, payload_hash])
    scope = "%s/%s/%s/aws4_request" % (date, region, service)
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(creq.encode("utf-8")).hexdigest()])
    sig = hmac.new(signing_key(secret, date, region, service), sts.encode("utf-8"), hashlib.sha256).hexdigest()
    return "AWS4-HMAC-SHA256 Credential=%s/%s, SignedHeaders=%s, Signature=%s" % (access_key, scope, sh, sig)


def split_s3(path):
    u = urlparse(str(path))
    if u.scheme.lower() not in ("s3", "s3a", "s3n"):
        raise ValueError("not an s3 path: %s" % path)
    return u.netloc, u.path.lstrip("/")


class S3Error(IOError):
    def __init__(self, status, body, what):
        super().__init__("S3 %s failed: HTTP %d %s" % (what, status, body[:300]))
        self.status = status


class S3ConfigError(RuntimeError):
    pass


class S3Client:
    def __init__(self, endpoint=None, region=None, access_key=None, secret_key=None, session_token=None,
                 timeout=60):
        self.region = region or os.environ.get("AWS_REGION") or os.environ.get("AWS_DEFAULT_REGION") or "us-east-1"
        ep = endpoint or os.environ.get("ZOO_S3_ENDPOINT") or os.environ.get("AWS_ENDPOINT_URL") or \
            "https://s3.%s.amazonaws.com" % self.region
        u = urlparse(ep)
        self.secure = u.scheme == "https"
        self.host = u.netloc
        self.access_key = access_key or os.environ.get("AWS_ACCESS_KEY_ID", "")
        self.secret_key = secret_key or os.environ.get("AWS_SECRET_ACCESS_KEY", "")
        self.session_token = session_token or os.environ.get("AWS_SESSION_TOKEN")
        self.timeout = timeout

    def _request(self, method, bucket, key="", query=None, body=b"", extra_headers=None, what="request"):
        if not self.access_key and not (os.environ.get("ZOO_S3_ENDPOINT") or os.environ.get("AWS_ENDPOINT_URL")):
            raise S3ConfigError("s3:// paths need AWS_ACCESS_KEY_ID / AWS_SECRET_ACCESS_KEY (and ZOO_S3_ENDPOINT "
                                "or AWS_ENDPOINT_URL for S3-compatible stores)")
        query = dict(query or {})
        uri = "/" + _uri_encode(bucket) + ("/" + _uri_encode(key) if key else "")
        payload_hash = hashlib.sha256(body).hexdigest()
        amz_date = datetime.datetime.now(datetime.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
        headers = {"host": self.host, "x-amz-date": amz_date, "x-amz-content-sha256": payload_hash}
        if self.session_token:
            headers["x-amz-security-token"] = self.session_token
        headers.update(extra_headers or {})
        if self.access_key:
            headers["Authorization"] = sign_v4(method, uri, query, {k: v for k, v in headers.items()},
                                               payload_hash, self.access_key, self.secret_key, self.region, amz_date)
        qs = "&".join("%s=%s" % (_uri_encode(k, False), _uri_encode(str(v), False)) for k, v in sorted(query.items()))
        conn_cls = http.client.HTTPSConnection if self.secure else http.client.HTTPConnection
        conn = conn_cls(self.host, timeout=self.timeout)
        try:
            conn.request(method, uri + ("?" + qs if qs else ""), body=body if body else None,
                         headers={k: v for k, v in headers.items() if k != "host"})
            resp = conn.getresponse()
            data = resp.read()
            return resp.status, data, dict(resp.getheaders())
        finally:
            conn.close()

    # -- objects
    def get(self, bucket, key, byte_range=None):
        h = {"Range": "bytes=%d-%d" % byte_range} if byte_range else None
        st, data, _ = self._request("GET", bucket, key, extra_headers=h, what="GET")
        if st not in (200, 206):
            raise S3Error(st, data, "GET s3://%s/%s" % (bucket, key))
        return data

    def put(self, bucket, key, data):
        st, body, _ = self._request("PUT", bucket, key, body=bytes(data), what="PUT")
        if st not in (200, 201):
            raise S3Error(st, body, "PUT s3://%s/%s" % (bucket, key))

    def head(self, bucket, key):
        st, _, hdrs = self._request("HEAD", bucket, key, what="HEAD")
        if st == 404:
            return None
        if st != 200:
            raise S3Error(st, b"", "HEAD s3://%s/%s" % (bucket, key))
        return hdrs

    def delete(self, bucket, key):
        st, body, _ = self._request("DELETE", bucket, key, what="DELETE")
        if st not in (200, 204, 404):
            raise S3Error(st, body, "DELETE s3://%s/%s" % (bucket, key))

    def list(self, bucket, prefix="", delimiter=None):
        """-> (object keys, common prefixes) under ``prefix`` (ListObjectsV2, paginated)."""
        keys, prefixes, token = [], [], None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if delimiter:
                q["delimiter"] = delimiter
            if token:
                q["continuation-token"] = token
            st, data, _ = self._request("GET", bucket, "", query=q, what="LIST")
            if st != 200:
                raise S3Error(st, data, "LIST s3://%s/%s" % (bucket, prefix))
            root = ET.fromstring(data)
            ns = root.tag[:root.tag.index("}") + 1] if root.tag.startswith("{") else ""
            keys += [c.findtext(ns + "Key") for c in root.findall(ns + "Contents")]
            prefixes += [c.findtext(ns + "Prefix") for c in root.findall(ns + "CommonPrefixes")]
            if root.findtext(ns + "IsTruncated", "false").lower() != "true":
                return keys, prefixes
            token = root.findtext(ns + "NextContinuationToken")


_CLIENT = []


def client():
    if not _CLIENT:
        _CLIENT.append(S3Client())
    return _CLIENT[0]


def reset_client():
    _CLIENT.clear()
