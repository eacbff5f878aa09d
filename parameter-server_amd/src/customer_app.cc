// customer_app.cc — Customer (reference src/internal/Customer.cpp:9-70) and
// SimpleApp (src/ps/SimpleApp.cpp).
#include <cstdlib>

#include "internal/PostOffice.h"
#include "internal/customer.h"
#include "ps/simple_app.h"

namespace ps {

Customer::Customer(int app_id, int customer_id, const ReceiveHandle& handle)
    : app_id_(app_id), customer_id_(customer_id), po_(PostOffice::Get()), receive_handle_(handle) {
  po_->AddCustomer(this);
  receive_thread_.reset(new std::thread(&Customer::ReceiveThread, this));
}

Customer::~Customer() {
  po_->RemoveCustomer(this);
  Message term;
  term.meta.control.cmd = Control::TERMINATE;
  term.meta.priority = -(1 << 30);  // after everything already queued
  receive_queue_.Push(term);
  receive_thread_->join();
}

int Customer::NewRequest(int receiver) {
  std::lock_guard<std::mutex> lk(tracker_mu_);
  int num = (int)po_->GetNodeIDs(receiver).size();
  tracker_.emplace_back(num, 0);
  return (int)tracker_.size() - 1;
}

int SpinMicros() {
  static const int us = [] {
    const char* e = std::getenv("PS_SPIN_US");
    return e ? std::atoi(e) : 250;
  }();
  return us;
}

void Customer::WaitRequest(int request_id) {
  {
    // spin while no request completes; re-check under the lock when one does
    uint64_t seen = completions_.load(std::memory_order_acquire);
    bool done;
    {
      std::lock_guard<std::mutex> lk(tracker_mu_);
      done = tracker_[request_id].first == tracker_[request_id].second;
    }
    if (done) return;
    SpinFor([&] {
      const uint64_t c = completions_.load(std::memory_order_acquire);
      if (c == seen) return false;
      seen = c;
      std::lock_guard<std::mutex> lk(tracker_mu_);
      done = tracker_[request_id].first == tracker_[request_id].second;
      return done;
    });
    if (done) return;
  }
  std::unique_lock<std::mutex> lk(tracker_mu_);
  while (tracker_[request_id].first != tracker_[request_id].second) {
    tracker_cond_.wait_for(lk, std::chrono::milliseconds(100));
    if (cluster::Aborted()) {
      lk.unlock();
      LOG(FATAL) << "request " << request_id << " abandoned: " << cluster::AbortReason();
    }
  }
}

int Customer::GetResponse(int request_id) {
  std::lock_guard<std::mutex> lk(tracker_mu_);
  return tracker_[request_id].second;
}

void Customer::ExpectMore(int request_id, int cnt) {
  std::lock_guard<std::mutex> lk(tracker_mu_);
  tracker_[request_id].first += cnt;
}

int Customer::NumExpected(int request_id) {
  std::lock_guard<std::mutex> lk(tracker_mu_);
  return tracker_[request_id].first;
}

void Customer::AddResponse(int request_id, int cnt) {
  std::lock_guard<std::mutex> lk(tracker_mu_);
  tracker_[request_id].second += cnt;
  if (tracker_[request_id].first == tracker_[request_id].second) {
    completions_.fetch_add(1, std::memory_order_release);
    tracker_cond_.notify_all();
  }
}

void Customer::ReceiveThread() {
  po_->BindThread();
  while (true) {
    Message msg = receive_queue_.WaitAndPop();
    if (msg.meta.control.cmd == Control::TERMINATE) break;
    try {
      receive_handle_(msg);
    } catch (const std::exception& e) {
      // a CHECK in a handle: the reference's uncaught PSError terminates the
      // process; here the job is aborted so every waiter throws instead
      cluster::Abort(std::string("handle of app ") + std::to_string(app_id_) + " threw: " + e.what());
      break;
    }
    if (!msg.meta.request) {
      std::lock_guard<std::mutex> lk(tracker_mu_);
      int r = msg.meta.timestamp;
      if (++tracker_[r].second == tracker_[r].first) {
        completions_.fetch_add(1, std::memory_order_release);
        tracker_cond_.notify_all();
      }
    }
  }
}

// ---------------------------------------------------------------------------

SimpleApp::SimpleApp() {
  request_handle_ = [](SimpleApp* app, const SimpleData& received) { app->Response(received); };
  response_handle_ = [](SimpleApp*, const SimpleData&) {};
}

SimpleApp::SimpleApp(int app_id, int customer_id) : SimpleApp() {
  app_id_ = app_id;
  customer_ = new Customer(app_id, customer_id, [this](const Message& m) { OnReceive(m); });
}

SimpleApp::~SimpleApp() {
  delete customer_;
  customer_ = nullptr;
}

int SimpleApp::Request(int request_head, const std::string& request_body, int receiver) {
  Message msg;
  msg.meta.head = request_head;
  msg.meta.body = request_body;
  msg.meta.request = true;
  msg.meta.simple_app = true;
  msg.meta.app_id = customer_->app_id();
  msg.meta.customer_id = customer_->customer_id();
  int request_id = customer_->NewRequest(receiver);
  msg.meta.timestamp = request_id;
  for (int id : PostOffice::Get()->GetNodeIDs(receiver)) {
    msg.meta.receiver = id;
    PostOffice::Get()->van()->Send(msg);
  }
  return request_id;
}

void SimpleApp::Response(const SimpleData& req, const std::string& response_body) {
  Message msg;
  msg.meta.head = req.head;
  msg.meta.body = response_body;
  msg.meta.request = false;
  msg.meta.simple_app = true;
  msg.meta.app_id = app_id_;
  msg.meta.customer_id = req.customer_id;
  msg.meta.timestamp = req.request_id;
  msg.meta.receiver = req.sender;
  PostOffice::Get()->van()->Send(msg);
}

void SimpleApp::Wait(int request_id) { customer_->WaitRequest(request_id); }

void SimpleApp::SetRequestHandle(const Handle& h) {
  CHECK(static_cast<bool>(h)) << "Handle shouldn't be empty";
  {
    std::lock_guard<std::mutex> lk(handle_mu_);
    request_handle_ = h;
    user_request_handle_ = true;
  }
  handle_cv_.notify_all();
}
void SimpleApp::SetResponseHandle(const Handle& h) {
  CHECK(static_cast<bool>(h)) << "Handle shouldn't be empty";
  std::lock_guard<std::mutex> lk(handle_mu_);
  response_handle_ = h;
}

void SimpleApp::OnReceive(const Message& msg) {
  SimpleData received{msg.meta.head, msg.meta.sender, msg.meta.customer_id, msg.meta.timestamp, msg.meta.body};
  Handle h;
  {
    std::unique_lock<std::mutex> lk(handle_mu_);
    if (msg.meta.request && !user_request_handle_)
      handle_cv_.wait_until(lk, created_ + std::chrono::seconds(1), [this] { return user_request_handle_; });
    h = msg.meta.request ? request_handle_ : response_handle_;
  }
  h(this, received);
}

}  // namespace ps
