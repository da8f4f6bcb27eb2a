// Event.cpp — see Event.h (reference interface: /root/reference/src/Event.cpp:9-52).
#include "Event.h"

Event::Event(int x, int y, double t, int p) : x_(x), y_(y), pol_(p), t_(t) {}
Event::Event() : x_(0), y_(0), pol_(0), t_(0.0) {}

bool Event::setX(int v) { x_ = v; return true; }
bool Event::setY(int v) { y_ = v; return true; }
bool Event::setStamp(double v) { t_ = v; return true; }
bool Event::setPolarity(int v) { pol_ = v; return true; }

int Event::getX() const { return x_; }
int Event::getY() const { return y_; }
double Event::getStamp() const { return t_; }
int Event::getPolarity() const { return pol_; }
