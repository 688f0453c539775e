// A move-only callable wrapper with inline storage.
//
// std::function keeps only 16 bytes inline (libstdc++), so a callback that captures a few
// values, such as the parked /api/hola-chaining request's continuation (connection, content,
// span, start time), costs one malloc and one free per call on the worker. InlineFunction
// stores a callable of up to N bytes inside itself; anything larger fails to compile rather
// than silently falling back to the heap. Move-only, so captures need not be copyable.
#pragma once
#include <cstddef>
#include <new>
#include <type_traits>
#include <utility>

namespace hola {

template <typename Sig, size_t N = 256>
class InlineFunction;

template <typename R, typename... A, size_t N>
class InlineFunction<R(A...), N> {
 public:
  InlineFunction() = default;
  InlineFunction(std::nullptr_t) {}  // NOLINT: implicit, like std::function
  template <typename F, typename D = std::decay_t<F>,
            typename = std::enable_if_t<!std::is_same_v<D, InlineFunction> && std::is_invocable_r_v<R, D&, A...>>>
  InlineFunction(F&& f) {  // NOLINT: implicit, like std::function
    static_assert(sizeof(D) <= N, "callable too large for this InlineFunction: raise N");
    static_assert(alignof(D) <= alignof(std::max_align_t), "over-aligned callable");
    ::new (static_cast<void*>(buf_)) D(std::forward<F>(f));
    ops_ = &kOps<D>;
  }
  InlineFunction(InlineFunction&& o) noexcept { take(o); }
  InlineFunction& operator=(InlineFunction&& o) noexcept {
    if (this != &o) {
      reset();
      take(o);
    }
    return *this;
  }
  InlineFunction& operator=(std::nullptr_t) noexcept {
    reset();
    return *this;
  }
  InlineFunction(const InlineFunction&) = delete;
  InlineFunction& operator=(const InlineFunction&) = delete;
  ~InlineFunction() { reset(); }

  explicit operator bool() const { return ops_ != nullptr; }
  R operator()(A... a) { return ops_->call(buf_, std::forward<A>(a)...); }
  void reset() noexcept {
    if (ops_) {
      ops_->destroy(buf_);
      ops_ = nullptr;
    }
  }

 private:
  struct Ops {
    R (*call)(void*, A&&...);
    void (*move)(void* dst, void* src) noexcept;  // move-constructs dst, destroys src
    void (*destroy)(void*) noexcept;
  };
  template <typename D>
  static constexpr Ops kOps = {
      [](void* p, A&&... a) -> R { return (*static_cast<D*>(p))(std::forward<A>(a)...); },
      [](void* dst, void* src) noexcept {
        ::new (dst) D(std::move(*static_cast<D*>(src)));
        static_cast<D*>(src)->~D();
      },
      [](void* p) noexcept { static_cast<D*>(p)->~D(); }};

  void take(InlineFunction& o) noexcept {
    if (!o.ops_) return;
    o.ops_->move(buf_, o.buf_);
    ops_ = o.ops_;
    o.ops_ = nullptr;
  }

  alignas(std::max_align_t) unsigned char buf_[N];
  const Ops* ops_ = nullptr;
};

}  // namespace hola
