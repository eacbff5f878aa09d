// ps/simple_app.h — head/body request-response app, the base of KVWorker and
// KVServer (reference src/ps/SimpleApp.{h,cpp}).
#pragma once
#include <functional>
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

 private:
  Handle request_handle_;
  Handle response_handle_;
};

}  // namespace ps
