#include "pto/http.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>

#include <chrono>
#include <cstring>

namespace pto {

// ------------------------------------------------------------------ helpers
bool Url::parse(const std::string& s, Url* out) {
  Url u;
  std::string rest = s;
  auto p = rest.find("://");
  if (p != std::string::npos) {
    u.scheme = rest.substr(0, p);
    rest = rest.substr(p + 3);
  }
  auto slash = rest.find('/');
  std::string hostport = slash == std::string::npos ? rest : rest.substr(0, slash);
  u.base_path = slash == std::string::npos ? "" : rest.substr(slash);
  while (!u.base_path.empty() && u.base_path.back() == '/') u.base_path.pop_back();
  u.port = u.scheme == "https" ? 443 : 80;
  if (!hostport.empty() && hostport[0] == '[') {  // [ipv6]:port
    auto rb = hostport.find(']');
    if (rb == std::string::npos) return false;
    u.host = hostport.substr(1, rb - 1);
    if (rb + 1 < hostport.size() && hostport[rb + 1] == ':') u.port = std::atoi(hostport.c_str() + rb + 2);
  } else {
    auto c = hostport.rfind(':');
    if (c != std::string::npos) {
      u.host = hostport.substr(0, c);
      u.port = std::atoi(hostport.c_str() + c + 1);
    } else {
      u.host = hostport;
    }
  }
  if (u.host.empty() || u.port <= 0) return false;
  *out = u;
  return true;
}

std::string url_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      o += (char)c;
    } else {
      o += '%';
      o += hex[c >> 4];
      o += hex[c & 15];
    }
  }
  return o;
}

std::string base64_decode(const std::string& in) {
  static int T[256];
  static bool init = false;
  if (!init) {
    for (int i = 0; i < 256; ++i) T[i] = -1;
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) T[(unsigned char)a[i]] = i;
    init = true;
  }
  std::string out;
  int val = 0, bits = -8;
  for (unsigned char c : in) {
    if (T[c] == -1) continue;
    val = (val << 6) + T[c];
    bits += 6;
    if (bits >= 0) {
      out += (char)((val >> bits) & 0xFF);
      bits -= 8;
    }
  }
  return out;
}

static double mono_now() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------------ connection
struct HttpClient::Conn {
  int fd = -1;
  SSL* ssl = nullptr;
  ~Conn() {
    if (ssl) {
      SSL_shutdown(ssl);
      SSL_free(ssl);
    }
    if (fd >= 0) ::close(fd);
  }
  // returns bytes read, 0 on EOF, -1 error, -2 timeout
  int read_some(char* buf, int n, double timeout_s) {
    if (ssl && SSL_pending(ssl) > 0) {
      int r = SSL_read(ssl, buf, n);
      return r > 0 ? r : -1;
    }
    struct pollfd p{fd, POLLIN, 0};
    int pr = ::poll(&p, 1, timeout_s < 0 ? -1 : (int)(timeout_s * 1000));
    if (pr == 0) return -2;
    if (pr < 0) return -1;
    if (ssl) {
      int r = SSL_read(ssl, buf, n);
      if (r > 0) return r;
      int e = SSL_get_error(ssl, r);
      if (e == SSL_ERROR_ZERO_RETURN) return 0;
      if (e == SSL_ERROR_WANT_READ) return -2;
      return -1;
    }
    ssize_t r = ::recv(fd, buf, (size_t)n, 0);
    return r < 0 ? -1 : (int)r;
  }
  bool write_all(const std::string& data) {
    size_t off = 0;
    while (off < data.size()) {
      int w;
      if (ssl) {
        w = SSL_write(ssl, data.data() + off, (int)(data.size() - off));
      } else {
        w = (int)::send(fd, data.data() + off, data.size() - off, MSG_NOSIGNAL);
      }
      if (w <= 0) return false;
      off += (size_t)w;
    }
    return true;
  }
};

static bool load_pem_ca(SSL_CTX* ctx, const std::string& pem) {
  BIO* bio = BIO_new_mem_buf(pem.data(), (int)pem.size());
  X509_STORE* store = SSL_CTX_get_cert_store(ctx);
  bool any = false;
  while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
    X509_STORE_add_cert(store, x);
    X509_free(x);
    any = true;
  }
  BIO_free(bio);
  ERR_clear_error();
  return any;
}

static std::string ssl_err(const char* what) {
  char buf[256];
  ERR_error_string_n(ERR_get_error(), buf, sizeof buf);
  ERR_clear_error();
  return std::string(what) + ": " + buf;
}

// Verification follows client-go: the server certificate must chain to the configured CA
// (kubeconfig certificate-authority[-data], the service-account ca.crt in-cluster, else the
// system store) AND name the host -- the URL's host, or tls-server-name when set; an IP
// literal is matched against the certificate's IP SANs.  A credential that fails to load
// is an error on every request (never a silent anonymous/unverified connection).
HttpClient::HttpClient(Url url, TlsConfig tls, std::string bearer_token, double timeout_s)
    : url_(std::move(url)), tls_(std::move(tls)), token_(std::move(bearer_token)), timeout_s_(timeout_s) {
  if (url_.scheme == "https") {
    SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
    if (tls_.insecure_skip_verify) {
      SSL_CTX_set_verify(ctx, SSL_VERIFY_NONE, nullptr);
    } else {
      SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
      if (!tls_.ca_file.empty() && SSL_CTX_load_verify_locations(ctx, tls_.ca_file.c_str(), nullptr) != 1)
        init_error_ = ssl_err(("cannot load CA file " + tls_.ca_file).c_str());
      if (!tls_.ca_data.empty() && !load_pem_ca(ctx, tls_.ca_data))
        init_error_ = "certificate-authority-data holds no PEM certificate";
      if (tls_.ca_file.empty() && tls_.ca_data.empty()) SSL_CTX_set_default_verify_paths(ctx);
    }
    if (!tls_.cert_file.empty() && SSL_CTX_use_certificate_chain_file(ctx, tls_.cert_file.c_str()) != 1)
      init_error_ = ssl_err(("cannot load client certificate " + tls_.cert_file).c_str());
    if (!tls_.key_file.empty() && SSL_CTX_use_PrivateKey_file(ctx, tls_.key_file.c_str(), SSL_FILETYPE_PEM) != 1)
      init_error_ = ssl_err(("cannot load client key " + tls_.key_file).c_str());
    if (!tls_.cert_data.empty()) {
      BIO* b = BIO_new_mem_buf(tls_.cert_data.data(), (int)tls_.cert_data.size());
      X509* x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr);
      if (x == nullptr || SSL_CTX_use_certificate(ctx, x) != 1) init_error_ = ssl_err("client-certificate-data");
      if (x) X509_free(x);
      BIO_free(b);
    }
    if (!tls_.key_data.empty()) {
      BIO* b = BIO_new_mem_buf(tls_.key_data.data(), (int)tls_.key_data.size());
      EVP_PKEY* k = PEM_read_bio_PrivateKey(b, nullptr, nullptr, nullptr);
      if (k == nullptr || SSL_CTX_use_PrivateKey(ctx, k) != 1) init_error_ = ssl_err("client-key-data");
      if (k) EVP_PKEY_free(k);
      BIO_free(b);
    }
    if (init_error_.empty() && (!tls_.cert_file.empty() || !tls_.cert_data.empty()) &&
        SSL_CTX_check_private_key(ctx) != 1)
      init_error_ = ssl_err("client certificate and key do not match");
    ssl_ctx_ = ctx;
  }
}

void HttpClient::set_bearer_token(std::string token) {
  std::lock_guard<std::mutex> g(token_mu_);
  token_ = std::move(token);
}

HttpClient::~HttpClient() {
  if (ssl_ctx_) SSL_CTX_free((SSL_CTX*)ssl_ctx_);
}

std::unique_ptr<HttpClient::Conn> HttpClient::connect(std::string* error, double timeout_s) {
  if (!init_error_.empty()) {
    *error = init_error_;
    return nullptr;
  }
  struct addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  std::string port = std::to_string(url_.port);
  int rc = getaddrinfo(url_.host.c_str(), port.c_str(), &hints, &res);
  if (rc != 0) {
    *error = std::string("resolve ") + url_.host + ": " + gai_strerror(rc);
    return nullptr;
  }
  auto conn = std::make_unique<Conn>();
  for (auto* ai = res; ai; ai = ai->ai_next) {
    int fd = ::socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
    if (fd < 0) continue;
    struct timeval tv{(time_t)timeout_s, (suseconds_t)((timeout_s - (int)timeout_s) * 1e6)};
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    if (::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) {
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      conn->fd = fd;
      break;
    }
    ::close(fd);
  }
  freeaddrinfo(res);
  if (conn->fd < 0) {
    *error = "connect " + url_.host + ":" + port + " failed: " + std::strerror(errno);
    return nullptr;
  }
  if (ssl_ctx_) {
    conn->ssl = SSL_new((SSL_CTX*)ssl_ctx_);
    SSL_set_fd(conn->ssl, conn->fd);
    const std::string& name = tls_.server_name.empty() ? url_.host : tls_.server_name;
    unsigned char ip[16];
    const bool is_ip = inet_pton(AF_INET, name.c_str(), ip) == 1 || inet_pton(AF_INET6, name.c_str(), ip) == 1;
    if (!is_ip) SSL_set_tlsext_host_name(conn->ssl, name.c_str());  // SNI carries DNS names only
    if (!tls_.insecure_skip_verify) {
      int ok;
      if (is_ip) {
        ok = X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(conn->ssl), name.c_str());
      } else {
        SSL_set_hostflags(conn->ssl, X509_CHECK_FLAG_NO_PARTIAL_WILDCARDS);
        ok = SSL_set1_host(conn->ssl, name.c_str());
      }
      if (ok != 1) {
        *error = "cannot set the expected server name " + name;
        return nullptr;
      }
    }
    if (SSL_connect(conn->ssl) != 1) {
      const long vr = SSL_get_verify_result(conn->ssl);
      std::string detail = vr != X509_V_OK ? X509_verify_cert_error_string(vr) : ssl_err("handshake");
      ERR_clear_error();
      *error = "TLS handshake with " + url_.host + " failed: " + detail;
      return nullptr;
    }
  }
  return conn;
}

std::string HttpClient::build_request(const std::string& method, const std::string& path,
                                      const std::string& body, const std::string& ctype,
                                      bool keepalive) {
  std::string req = method + " " + url_.base_path + path + " HTTP/1.1\r\n";
  req += "Host: " + url_.host + ":" + std::to_string(url_.port) + "\r\n";
  req += "User-Agent: pytorch-operator/v1 (mi355x-native)\r\n";
  req += "Accept: application/json\r\n";
  {
    std::lock_guard<std::mutex> g(token_mu_);
    if (!token_.empty()) req += "Authorization: Bearer " + token_ + "\r\n";
  }
  if (!body.empty() || method == "POST" || method == "PUT" || method == "PATCH") {
    req += "Content-Type: " + ctype + "\r\n";
    req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  }
  req += keepalive ? "Connection: keep-alive\r\n" : "Connection: close\r\n";
  req += "\r\n";
  req += body;
  return req;
}

namespace {
// Incremental HTTP/1.1 response reader (status line, headers, identity/chunked body).
struct RespReader {
  std::string buf;
  bool headers_done = false, chunked = false;
  long content_length = -1;
  int status = 0;
  std::map<std::string, std::string> headers;
  size_t body_consumed = 0;

  bool parse_headers() {
    auto end = buf.find("\r\n\r\n");
    if (end == std::string::npos) return false;
    std::string head = buf.substr(0, end);
    buf.erase(0, end + 4);
    size_t pos = head.find("\r\n");
    std::string status_line = head.substr(0, pos);
    auto sp = status_line.find(' ');
    status = sp == std::string::npos ? 0 : std::atoi(status_line.c_str() + sp + 1);
    while (pos != std::string::npos) {
      size_t next = head.find("\r\n", pos + 2);
      std::string line = head.substr(pos + 2, next == std::string::npos ? std::string::npos : next - pos - 2);
      auto c = line.find(':');
      if (c != std::string::npos) {
        std::string k = line.substr(0, c), v = line.substr(c + 1);
        while (!v.empty() && v[0] == ' ') v.erase(0, 1);
        for (auto& ch : k) ch = (char)std::tolower((unsigned char)ch);
        headers[k] = v;
      }
      pos = next;
    }
    auto te = headers.find("transfer-encoding");
    chunked = te != headers.end() && te->second.find("chunked") != std::string::npos;
    auto cl = headers.find("content-length");
    if (cl != headers.end()) content_length = std::atol(cl->second.c_str());
    headers_done = true;
    return true;
  }

  // Extract decoded body bytes available so far; done=true when the body is complete.
  std::string take_body(bool* done, bool eof) {
    std::string out;
    *done = false;
    if (!chunked) {
      out.swap(buf);
      body_consumed += out.size();
      if (content_length >= 0 && (long)body_consumed >= content_length) *done = true;
      if (eof) *done = true;
      return out;
    }
    while (true) {
      auto le = buf.find("\r\n");
      if (le == std::string::npos) break;
      long n = std::strtol(buf.substr(0, le).c_str(), nullptr, 16);
      if (n == 0) {
        *done = true;
        buf.clear();
        break;
      }
      if (buf.size() < le + 2 + (size_t)n + 2) break;
      out.append(buf, le + 2, (size_t)n);
      buf.erase(0, le + 2 + (size_t)n + 2);
    }
    if (eof) *done = true;
    return out;
  }
};
}  // namespace

HttpResponse HttpClient::request(const std::string& method, const std::string& path,
                                 const std::string& body, const std::string& ctype) {
  HttpResponse resp;
  auto conn = connect(&resp.error, timeout_s_);
  if (!conn) return resp;
  if (!conn->write_all(build_request(method, path, body, ctype, false))) {
    resp.error = "write failed";
    return resp;
  }
  RespReader rr;
  char buf[16384];
  double deadline = mono_now() + timeout_s_;
  bool done = false;
  while (!done) {
    double left = deadline - mono_now();
    if (left <= 0) {
      resp.error = "timeout";
      return resp;
    }
    int n = conn->read_some(buf, sizeof buf, left);
    if (n == -2) continue;
    if (n < 0) {
      resp.error = "read failed";
      return resp;
    }
    bool eof = n == 0;
    if (n > 0) rr.buf.append(buf, (size_t)n);
    if (!rr.headers_done && !rr.parse_headers()) {
      if (eof) {
        resp.error = "connection closed before headers";
        return resp;
      }
      continue;
    }
    resp.body += rr.take_body(&done, eof);
    if (rr.content_length == 0) done = true;
  }
  resp.status = rr.status;
  resp.headers = rr.headers;
  return resp;
}

int HttpClient::stream_lines(const std::string& path, const std::function<bool(const std::string&)>& on_line,
                             const std::atomic<bool>* stop, double idle_timeout_s, std::string* error) {
  auto conn = connect(error, timeout_s_);
  if (!conn) return 0;
  if (!conn->write_all(build_request("GET", path, "", "application/json", false))) {
    *error = "write failed";
    return 0;
  }
  RespReader rr;
  std::string pending;
  char buf[16384];
  double last = mono_now();
  bool done = false;
  while (!done) {
    if (stop && stop->load()) return rr.status;
    int n = conn->read_some(buf, sizeof buf, 0.25);
    if (n == -2) {
      if (idle_timeout_s > 0 && mono_now() - last > idle_timeout_s) return rr.status;
      continue;
    }
    if (n < 0) {
      *error = "read failed";
      return rr.status;
    }
    last = mono_now();
    bool eof = n == 0;
    if (n > 0) rr.buf.append(buf, (size_t)n);
    if (!rr.headers_done && !rr.parse_headers()) {
      if (eof) return 0;
      continue;
    }
    pending += rr.take_body(&done, eof);
    if (rr.status != 200) {
      if (done) {
        if (!pending.empty()) on_line(pending);
        return rr.status;
      }
      continue;
    }
    size_t nl;
    while ((nl = pending.find('\n')) != std::string::npos) {
      std::string line = pending.substr(0, nl);
      pending.erase(0, nl + 1);
      if (!line.empty() && !on_line(line)) return rr.status;
    }
  }
  if (!pending.empty()) on_line(pending);
  return rr.status;
}

// ------------------------------------------------------------------ server
HttpServer::HttpServer(std::string bind_addr, int port, Handler h)
    : addr_(std::move(bind_addr)), port_(port), handler_(std::move(h)) {}

HttpServer::~HttpServer() { stop(); }

bool HttpServer::start(std::string* error) {
  fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  struct sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port_);
  sa.sin_addr.s_addr = addr_.empty() ? INADDR_ANY : inet_addr(addr_.c_str());
  if (::bind(fd_, (struct sockaddr*)&sa, sizeof sa) != 0 || ::listen(fd_, 64) != 0) {
    *error = std::string("bind/listen failed: ") + std::strerror(errno);
    ::close(fd_);
    fd_ = -1;
    return false;
  }
  socklen_t len = sizeof sa;
  getsockname(fd_, (struct sockaddr*)&sa, &len);
  port_ = ntohs(sa.sin_port);
  th_ = std::thread([this] { loop(); });
  return true;
}

void HttpServer::stop() {
  if (stop_.exchange(true)) return;
  if (fd_ >= 0) {
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
  }
  if (th_.joinable()) th_.join();
}

void HttpServer::loop() {
  while (!stop_.load()) {
    struct pollfd p{fd_, POLLIN, 0};
    if (::poll(&p, 1, 200) <= 0) continue;
    int c = ::accept(fd_, nullptr, nullptr);
    if (c < 0) continue;
    std::string req;
    char buf[8192];
    while (req.find("\r\n\r\n") == std::string::npos) {
      struct pollfd q{c, POLLIN, 0};
      if (::poll(&q, 1, 2000) <= 0) break;
      ssize_t n = ::recv(c, buf, sizeof buf, 0);
      if (n <= 0) break;
      req.append(buf, (size_t)n);
    }
    std::string method, path;
    {
      auto sp1 = req.find(' ');
      auto sp2 = req.find(' ', sp1 + 1);
      if (sp1 != std::string::npos && sp2 != std::string::npos) {
        method = req.substr(0, sp1);
        path = req.substr(sp1 + 1, sp2 - sp1 - 1);
      }
    }
    std::string body;
    auto he = req.find("\r\n\r\n");
    if (he != std::string::npos) body = req.substr(he + 4);
    Reply r = method.empty() ? Reply{400, "text/plain", "bad request\n"} : handler_(method, path, body);
    std::string out = "HTTP/1.1 " + std::to_string(r.status) + (r.status == 200 ? " OK" : " Error") + "\r\n";
    out += "Content-Type: " + r.content_type + "\r\n";
    out += "Content-Length: " + std::to_string(r.body.size()) + "\r\nConnection: close\r\n\r\n" + r.body;
    size_t off = 0;
    while (off < out.size()) {
      ssize_t w = ::send(c, out.data() + off, out.size() - off, MSG_NOSIGNAL);
      if (w <= 0) break;
      off += (size_t)w;
    }
    ::close(c);
  }
}

}  // namespace pto
