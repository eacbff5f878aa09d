// ps/simple_app.h — head/body request-response app, the base of KVWorker and
// KVServer (reference src/ps/SimpleApp.{h,cpp}).
#pragma once
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>

#include "internal/customer.h"
#include "internal/message.h"

namespace ps {

struct SimpleData {
  int head;
  int sender;
  int customer_id;
  int request_id;
  std::string body;
};

class SimpleApp {
 public:
  using Handle = std::function<void(SimpleApp* app, const SimpleData& received)>;

  SimpleApp(int app_id, int customer_id);
  virtual ~SimpleApp();

  /* send head/body to a node or group; returns the request id */
  virtual int Request(int request_head, const std::string& request_body, int receiver);
  void Response(const SimpleData& request_msg, const std::string& response_body = "");
  virtual void Wait(int request_id);
  void SetRequestHandle(const Handle& request_handle);
  void SetResponseHandle(const Handle& response_handle);
  virtual Customer* GetCustomer() { return customer_; }

 protected:
  SimpleApp();
  virtual void OnReceive(const Message& msg);
  Customer* customer_{nullptr};
  int app_id_ = 0;  // known before customer_ is, which may already dispatch

 private:
  // The handles are swapped by the program's thread while the customer thread
  // may be calling them: guarded.  A request that arrives within the first
  // second of the app, before the program installed its handle, waits for it
  // (the program's next statement after the constructor, as in
  // test_simple_app.cpp) instead of taking the default one.
  std::mutex handle_mu_;
  std::condition_variable handle_cv_;
  bool user_request_handle_ = false;
  std::chrono::steady_clock::time_point created_ = std::chrono::steady_clock::now();
  Handle request_handle_;
  Handle response_handle_;
};

}  // namespace ps
