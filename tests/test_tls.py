"""TLS and authentication against an HTTPS API server (CPU).

The reference builds its clients with client-go (tf-operator k8sutil.go:44-68,
cmd/pytorch-operator.v1/app/server.go:85-99): the server certificate must chain to the
kubeconfig CA *and* name the host; credentials are bearer tokens, client certificates or
exec plugins.  Here the fake API server serves HTTPS with a test CA made by the openssl CLI
and requires a token or a CA-signed client certificate (401 otherwise); the native C++
operator and the Python SDK must connect with every credential kind, honour
``tls-server-name``, and refuse a certificate issued for another host.
"""
import json
import os
import ssl
import subprocess
import sys
import time
import urllib.request

import pytest

from pytorch_operator_amd.cluster.fake_apiserver import FakeApiServer
from pytorch_operator_amd.cluster.local import free_port, operator_binary
from kubeflow.pytorchjob.rest import PYTORCHJOBS, ApiException, KubeRest, load_kube_config

TOKEN = "s3cret-operator-token"


def _openssl(*args, cwd):
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True)


def _leaf(d, name, cn, san, ca="ca", client=False):
    _openssl("req", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{name}.key", "-subj", f"/CN={cn}",
             "-out", f"{name}.csr", cwd=d)
    ext = f"{name}.ext"
    with open(os.path.join(d, ext), "w") as f:
        f.write("basicConstraints=CA:FALSE\n")
        f.write(f"extendedKeyUsage={'clientAuth' if client else 'serverAuth'}\n")
        if san:
            f.write(f"subjectAltName={san}\n")
    _openssl("x509", "-req", "-in", f"{name}.csr", "-CA", f"{ca}.crt", "-CAkey", f"{ca}.key",
             "-CAcreateserial", "-days", "2", "-sha256", "-extfile", ext, "-out", f"{name}.crt", cwd=d)
    return os.path.join(d, f"{name}.crt"), os.path.join(d, f"{name}.key")


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("pki"))
    _openssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-subj", "/CN=test-ca",
             "-days", "2", "-out", "ca.crt", cwd=d)
    p = {"dir": d, "ca": os.path.join(d, "ca.crt")}
    p["server"] = _leaf(d, "server", "kube-apiserver", "DNS:localhost,IP:127.0.0.1")
    p["wrong"] = _leaf(d, "wrong", "other", "DNS:api.other.example")
    p["client"] = _leaf(d, "client", "system:serviceaccount:kubeflow:pytorch-operator", None, client=True)
    # a client certificate from a CA the server does not trust
    _openssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "rogue.key", "-subj", "/CN=rogue-ca",
             "-days", "2", "-out", "rogue.crt", cwd=d)
    p["rogue_client"] = _leaf(d, "rclient", "intruder", None, ca="rogue", client=True)
    return p


def _server(pki, cert="server", url_host=None):
    crt, key = pki[cert]
    api = FakeApiServer(tls={"cert": crt, "key": key, "client_ca": pki["ca"]}, tokens={TOKEN},
                        url_host=url_host).start()
    api.install_crds()
    return api


def _exec_plugin_script(d, token):
    p = os.path.join(d, f"cred-{token[:6]}.py")
    with open(p, "w") as f:
        f.write("import json, os\n"
                "info = json.loads(os.environ['KUBERNETES_EXEC_INFO'])\n"
                f"print(json.dumps({{'apiVersion': info['apiVersion'], 'kind': 'ExecCredential', "
                f"'status': {{'token': {token!r}}}}}))\n")
    return {"apiVersion": "client.authentication.k8s.io/v1", "command": sys.executable, "args": [p]}


# ---------------------------------------------------------------------------- SDK (Python)
def _sdk(api, tmp_path, **kw):
    kc = api.write_kubeconfig(str(tmp_path / f"kc-{time.monotonic_ns()}.json"), **kw)
    return KubeRest(load_kube_config(kc), timeout=10)


def test_sdk_token_over_verified_tls_ip_and_dns(pki, tmp_path):
    api = _server(pki)
    try:
        assert "items" in _sdk(api, tmp_path, token=TOKEN, ca_file=pki["ca"]).list(PYTORCHJOBS, "default")
        dns = f"https://localhost:{api.port}"
        assert "items" in _sdk(api, tmp_path, token=TOKEN, ca_file=pki["ca"], server=dns).list(PYTORCHJOBS, "default")
    finally:
        api.stop()


def test_sdk_rejects_wrong_host_and_unknown_ca(pki, tmp_path):
    api = _server(pki, cert="wrong")
    try:
        with pytest.raises(ssl.SSLCertVerificationError):
            _sdk(api, tmp_path, token=TOKEN, ca_file=pki["ca"]).list(PYTORCHJOBS, "default")
        # tls-server-name: the certificate's name instead of the URL host
        r = _sdk(api, tmp_path, token=TOKEN, ca_file=pki["ca"], tls_server_name="api.other.example")
        assert "items" in r.list(PYTORCHJOBS, "default")
    finally:
        api.stop()
    api = _server(pki)
    try:
        with pytest.raises(ssl.SSLCertVerificationError):  # no CA given: system store only
            _sdk(api, tmp_path, token=TOKEN).list(PYTORCHJOBS, "default")
    finally:
        api.stop()


def test_sdk_authentication_kinds(pki, tmp_path):
    api = _server(pki)
    try:
        with pytest.raises(ApiException) as e:
            _sdk(api, tmp_path, token="wrong-token", ca_file=pki["ca"]).list(PYTORCHJOBS, "default")
        assert e.value.status == 401
        with pytest.raises(ApiException) as e:
            _sdk(api, tmp_path, token=None, ca_file=pki["ca"]).list(PYTORCHJOBS, "default")
        assert e.value.status == 401
        crt, key = pki["client"]
        assert "items" in _sdk(api, tmp_path, token=None, ca_file=pki["ca"], client_cert=crt,
                               client_key=key).list(PYTORCHJOBS, "default")
        rcrt, rkey = pki["rogue_client"]
        with pytest.raises((ApiException, ssl.SSLError, ConnectionError)):
            _sdk(api, tmp_path, token=None, ca_file=pki["ca"], client_cert=rcrt,
                 client_key=rkey).list(PYTORCHJOBS, "default")
        r = _sdk(api, tmp_path, token=None, ca_file=pki["ca"], exec_plugin=_exec_plugin_script(pki["dir"], TOKEN))
        assert r.config.token == TOKEN and "items" in r.list(PYTORCHJOBS, "default")
    finally:
        api.stop()


# ---------------------------------------------------------------------------- operator (C++)
def _run_operator(api, tmp_path, **kw):
    kc = api.write_kubeconfig(str(tmp_path / f"op-kc-{time.monotonic_ns()}.json"), **kw)
    port = free_port()
    log = open(tmp_path / f"op-{port}.log", "wb")
    env = dict(os.environ, KUBEFLOW_NAMESPACE="kubeflow")
    env.pop("KUBECONFIG", None)
    p = subprocess.Popen([operator_binary(), "--kubeconfig", kc, f"--monitoring-port={port}",
                          "--json-log-format=false"], env=env, stdout=log, stderr=subprocess.STDOUT,
                         start_new_session=True)
    return p, port, tmp_path / f"op-{port}.log"


def _is_leader(port):
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=2) as r:
            for line in r.read().decode().splitlines():
                if line.startswith("pytorch_operator_is_leader "):
                    return float(line.split()[1]) >= 1
    except OSError:
        return False
    return False


def _stop(p):
    p.terminate()
    try:
        p.wait(10)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()


def _expect_leader(p, port, log, timeout=20.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if _is_leader(port):
            return
        assert p.poll() is None, log.read_text()[-2000:]
        time.sleep(0.1)
    raise AssertionError("operator never became leader:\n" + log.read_text()[-3000:])


@pytest.mark.parametrize("mode", ["token-ip", "token-dns", "client-cert", "exec-plugin", "tls-server-name"])
def test_operator_connects_over_tls(pki, tmp_path, mode):
    api = _server(pki, cert="wrong" if mode == "tls-server-name" else "server")
    kw = {"ca_file": pki["ca"], "token": TOKEN}
    if mode == "token-dns":
        kw["server"] = f"https://localhost:{api.port}"
    elif mode == "client-cert":
        kw.update(token=None, client_cert=pki["client"][0], client_key=pki["client"][1])
    elif mode == "exec-plugin":
        kw.update(token=None, exec_plugin=_exec_plugin_script(pki["dir"], TOKEN))
    elif mode == "tls-server-name":
        kw["tls_server_name"] = "api.other.example"
    try:
        p, port, log = _run_operator(api, tmp_path, **kw)
        try:
            _expect_leader(p, port, log)
            assert api.store.request_count > 0
        finally:
            _stop(p)
    finally:
        api.stop()


@pytest.mark.parametrize("case", ["wrong-host", "wrong-ip-san", "untrusted-ca", "bad-token"])
def test_operator_refuses_bad_peer_or_credentials(pki, tmp_path, case):
    """A certificate for another host (or from a CA not configured) must never be accepted,
    and a rejected token must not be treated as a connection: the operator keeps retrying
    and never becomes leader."""
    api = _server(pki, cert="wrong" if case in ("wrong-host", "wrong-ip-san") else "server")
    kw = {"ca_file": pki["ca"], "token": TOKEN}
    if case == "wrong-host":
        kw["server"] = f"https://localhost:{api.port}"
    elif case == "untrusted-ca":
        kw["ca_file"] = os.path.join(pki["dir"], "rogue.crt")
    elif case == "bad-token":
        kw["token"] = "nope"
    try:
        p, port, log = _run_operator(api, tmp_path, **kw)
        try:
            time.sleep(3.0)
            assert not _is_leader(port)
        finally:
            _stop(p)
        text = log.read_text()
        if case == "wrong-host":
            assert "hostname mismatch" in text, text[-2000:]
        elif case == "wrong-ip-san":
            assert "IP address mismatch" in text, text[-2000:]
        elif case == "untrusted-ca":
            assert "TLS handshake" in text, text[-2000:]
        else:
            assert "Unauthorized" in text, text[-2000:]
    finally:
        api.stop()


def test_operator_rejects_unloadable_credentials(pki, tmp_path):
    """A kubeconfig whose client key does not match its certificate is an error on every
    request -- never a silent anonymous connection."""
    api = _server(pki)
    try:
        p, port, log = _run_operator(api, tmp_path, ca_file=pki["ca"], token=None,
                                     client_cert=pki["client"][0], client_key=pki["server"][1])
        try:
            time.sleep(2.0)
            assert not _is_leader(port)
        finally:
            _stop(p)
        assert "key values mismatch" in log.read_text() or "do not match" in log.read_text()
    finally:
        api.stop()


# ---------------------------------------------------------------------------- exec plugin hygiene
def test_sdk_cert_only_exec_plugin_runs_once_and_reuses_one_key_file(pki, tmp_path):
    """A plugin that returns only a client certificate is not rerun on every request (the
    credential check looks at any credential, not just a token), and its key lands in one
    private file per Configuration, rewritten in place."""
    from kubeflow.pytorchjob.configuration import ExecPlugin, Configuration
    crt, key = pki["client"]
    counter = tmp_path / "runs"
    script = tmp_path / "cert_plugin.py"
    script.write_text(
        "import json, os, sys\n"
        f"open({str(counter)!r}, 'a').write('x')\n"
        f"crt = open({crt!r}).read(); key = open({key!r}).read()\n"
        "print(json.dumps({'apiVersion': 'client.authentication.k8s.io/v1', 'kind': 'ExecCredential',"
        " 'status': {'clientCertificateData': crt, 'clientKeyData': key}}))\n")
    cfg = Configuration(host="https://127.0.0.1:1", exec_plugin=ExecPlugin(command=sys.executable, args=[str(script)]))
    cfg.refresh_credentials(force=True)
    first = (cfg.cert_file, cfg.key_file)
    for _ in range(5):
        cfg.refresh_credentials()
    assert counter.read_text() == "x"  # ran once
    assert os.stat(cfg.key_file).st_mode & 0o077 == 0
    cfg.refresh_credentials(force=True)  # a forced refresh rewrites the same two files
    assert (cfg.cert_file, cfg.key_file) == first and counter.read_text() == "xx"
    assert open(cfg.key_file).read() == open(key).read()
    # the pair lives in a private 0700 directory (no predictable names in the shared
    # temp dir that another local user could pre-create), rewritten through mkstemp temp files
    d = os.path.dirname(cfg.key_file)
    assert os.path.dirname(cfg.cert_file) == d and os.stat(d).st_mode & 0o777 == 0o700
    assert sorted(os.listdir(d)) == ["client.crt", "client.key"]


def test_operator_kills_a_hanging_exec_plugin(pki, tmp_path):
    """An exec credential plugin that never exits is killed at the deadline (here
    PTO_EXEC_PLUGIN_TIMEOUT_S=2) instead of blocking the operator forever in waitpid."""
    api = _server(pki)
    pidfile = tmp_path / "plugin.pid"
    script = tmp_path / "hang.py"
    script.write_text(f"import os, time\nopen({str(pidfile)!r}, 'w').write(str(os.getpid()))\ntime.sleep(600)\n")
    kc = api.write_kubeconfig(str(tmp_path / "kc-hang.json"), ca_file=pki["ca"], token=None,
                              exec_plugin={"apiVersion": "client.authentication.k8s.io/v1",
                                           "command": sys.executable, "args": [str(script)]})
    env = dict(os.environ, KUBEFLOW_NAMESPACE="kubeflow", PTO_EXEC_PLUGIN_TIMEOUT_S="2")
    env.pop("KUBECONFIG", None)
    log = tmp_path / "op-hang.log"
    try:
        t0 = time.time()
        with open(log, "wb") as lf:
            p = subprocess.Popen([operator_binary(), "--kubeconfig", kc, f"--monitoring-port={free_port()}",
                                  "--json-log-format=false"], env=env, stdout=lf, stderr=subprocess.STDOUT,
                                 start_new_session=True)
        try:
            p.wait(30)
        except subprocess.TimeoutExpired:
            _stop(p)
            raise AssertionError("operator blocked on the hung plugin:\n" + log.read_text()[-2000:])
        assert time.time() - t0 < 25
        assert p.returncode != 0
        assert "timed out" in log.read_text(), log.read_text()[-2000:]
        pid = int(pidfile.read_text())
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)  # killed and reaped
    finally:
        api.stop()
