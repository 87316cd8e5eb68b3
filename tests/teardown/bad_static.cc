// Negative control of tests/test_teardown.py: a library named like the
// product whose static object's destructor calls the HIP runtime -- the
// pattern the test must catch.
extern "C" int hipFree(void *);
namespace {
struct CallsHipAtExit {
    ~CallsHipAtExit() { hipFree(nullptr); }
} g_bad;
}  // namespace
extern "C" int lvgpu_bad_probe(void) { return 0; }
