// Minimal HTTP/1.1 client (plain TCP or TLS via OpenSSL) and server.
//
// The client is what the operator uses to talk to the Kubernetes API server
// (the reference uses client-go); it supports bearer tokens, client
// certificates, custom CAs, chunked transfer decoding and line-streamed
// responses for `?watch=true`.  The server backs the /metrics endpoint
// (reference: promhttp on --monitoring-port, cmd/pytorch-operator.v1/main.go:31-40).
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace pto {

struct Url {
  std::string scheme = "http", host = "127.0.0.1", base_path;
  int port = 80;
  static bool parse(const std::string& s, Url* out);
};

struct TlsConfig {
  std::string ca_file, cert_file, key_file;
  std::string ca_data, cert_data, key_data;  // PEM (kubeconfig *-data, base64-decoded)
  std::string server_name;  // kubeconfig tls-server-name: name checked instead of the URL host
  bool insecure_skip_verify = false;
};

struct HttpResponse {
  int status = 0;  // 0: transport error (see error)
  std::map<std::string, std::string> headers;  // lower-cased names
  std::string body;
  std::string error;
};

class HttpClient {
 public:
  HttpClient(Url url, TlsConfig tls = {}, std::string bearer_token = "", double timeout_s = 30.0);
  ~HttpClient();

  HttpResponse request(const std::string& method, const std::string& path,
                       const std::string& body = "", const std::string& content_type = "application/json");

  // Streams the response body line by line (watch).  on_line returns false to stop.
  // `stop` is polled between reads.  Returns the status (0 on transport error).
  int stream_lines(const std::string& path, const std::function<bool(const std::string&)>& on_line,
                   const std::atomic<bool>* stop, double idle_timeout_s, std::string* error);

  const Url& url() const { return url_; }
  // Replace the bearer token (exec-plugin credential refresh); thread-safe.
  void set_bearer_token(std::string token);

 private:
  struct Conn;
  std::unique_ptr<Conn> connect(std::string* error, double timeout_s);
  std::string build_request(const std::string& method, const std::string& path,
                            const std::string& body, const std::string& content_type, bool keepalive);

  Url url_;
  std::string init_error_;  // TLS material that failed to load (reported per request)
  TlsConfig tls_;
  std::string token_;
  mutable std::mutex token_mu_;
  double timeout_s_;
  void* ssl_ctx_ = nullptr;  // SSL_CTX*
};

// Tiny threaded HTTP server: handler(method, path, body) -> (status, content_type, body).
class HttpServer {
 public:
  struct Reply {
    int status = 200;
    std::string content_type = "text/plain; charset=utf-8";
    std::string body;
  };
  using Handler = std::function<Reply(const std::string& method, const std::string& path,
                                      const std::string& body)>;
  HttpServer(std::string bind_addr, int port, Handler h);
  ~HttpServer();
  bool start(std::string* error);  // binds; port 0 picks a free port
  void stop();
  int port() const { return port_; }

 private:
  void loop();
  std::string addr_;
  int port_;
  Handler handler_;
  int fd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread th_;
};

std::string url_encode(const std::string& s);
std::string base64_decode(const std::string& in);

}  // namespace pto
